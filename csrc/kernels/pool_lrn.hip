// pool_lrn.hip - NHWC pooling (max / avg / maxabs) and local response
// normalisation across channels, forward and backward, for gfx950.
//
// Replaces the (absent) Znicz pooling / gd_pooling / normalization kernels
// (docs/OPS.md).  Layout is NHWC so the channel vector of a
// pixel is contiguous: pooling threads own 8 channels (one 16-B bf16 load),
// LRN waves own one pixel and stage its channels in LDS.  Pooling backward is
// a deterministic GATHER (each input element sums the windows that chose it)
// instead of atomics.
#include "fp8_common.h"
#include "hvk_common.h"

using namespace hvk;

namespace {
// 2^x as the bare v_exp_f32: the LRN exponents are (-beta [- 1]) log2(s)
// with s >= k > 0, and denormal results flush to zero in these kernels
// anyway (-fgpu-flush-denormals-to-zero), so the library exp2f's range
// rescaling (a second v_exp plus compare / select / multiply per call) buys
// nothing
__device__ __forceinline__ float ex2(float x) {
  return __builtin_amdgcn_exp2f(x);
}

inline int grid_for(long long n, int per_block = 256) {
  long long g = (n + per_block - 1) / per_block;
  if (g > 16384) g = 16384;
  return g < 1 ? 1 : (int)g;
}

enum PoolMode { POOL_MAX = 0, POOL_AVG = 1, POOL_MAXABS = 2 };

// one thread = one output pixel x 8 channels (C % 8 == 0) or x 1 channel
template <int VEC>
__global__ void pool_fwd_kernel(const uint16_t* x, uint16_t* y, int* argmax,
                                int N, int H, int W, int C, int OH, int OW,
                                int ky, int kx, int sy, int sx, int pt, int pl,
                                int mode, FastDiv fCV, FastDiv fOW,
                                FastDiv fOH) {
  const int CV = C / VEC;
  const int total = N * OH * OW * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const int cv = cvu, ow = owu, n = nu, oh = ohu;
    int h0 = oh * sy - pt, w0 = ow * sx - pl;
    int h1 = min(h0 + ky, H), w1 = min(w0 + kx, W);
    h0 = max(h0, 0);
    w0 = max(w0, 0);
    float best[VEC], sum[VEC];
    int bidx[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) { best[q] = -INFINITY; sum[q] = 0.f; bidx[q] = -1; }
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        int off = ((n * H + h) * W + w) * C + cv * VEC;
        uint16_t v[VEC];
        if (VEC == 8) *(uint4*)v = *(const uint4*)(x + off);
        else if (VEC > 1) __builtin_memcpy(v, x + off, VEC * 2);
        else v[0] = x[off];
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          float f = bf2f(v[q]);
          if (mode == POOL_AVG) {
            sum[q] += f;
          } else {
            float key = mode == POOL_MAXABS ? fabsf(f) : f;
            float bk = mode == POOL_MAXABS ? fabsf(best[q]) : best[q];
            if (bidx[q] < 0 || key > bk) { best[q] = f; bidx[q] = off + q; }
          }
        }
      }
    int cnt = (h1 - h0) * (w1 - w0);
    uint16_t o[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      o[q] = f2bf(mode == POOL_AVG ? sum[q] / (float)max(cnt, 1) : best[q]);
    int yo = pix * C + cv * VEC;
    if (VEC == 8) *(uint4*)(y + yo) = *(uint4*)o;
    else if (VEC > 1) __builtin_memcpy(y + yo, o, VEC * 2);
    else y[yo] = o[0];
    if (argmax && mode != POOL_AVG) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) argmax[yo + q] = bidx[q];
    }
  }
}


// 3x3 windows, 8 channels per lane: all nine 16-B loads issued up front
// (clamped addresses + validity masks), argmax stored as two int4s.
template <int MODE>
__global__ void pool_fwd3_kernel(const uint16_t* __restrict__ x,
                                 uint16_t* __restrict__ y,
                                 int* __restrict__ argmax, int N, int H,
                                 int W, int C, int OH, int OW, int sy, int sx,
                                 int pt, int pl, FastDiv fCV,
                                 FastDiv fOW, FastDiv fOH) {
  constexpr int mode = MODE;
  const int CV = C >> 3;
  const int total = N * OH * OW * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const int h0 = (int)ohu * sy - pt, w0 = (int)owu * sx - pl;
    const long long img = (long long)nu * H * W * C + cvu * 8;
    uint4 v[9];
    int off[9];
    bool ok[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int h = h0 + i / 3, w = w0 + i % 3;
      ok[i] = h >= 0 && h < H && w >= 0 && w < W;
      const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1);
      off[i] = (hc * W + wc) * C;
      v[i] = *(const uint4*)(x + img + off[i]);
    }
    float best[8], sum[8];
    int bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { best[q] = -INFINITY; sum[q] = 0.f; bi[q] = -1; }
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      if (!ok[i]) continue;
      ++cnt;
      const uint16_t* hv = (const uint16_t*)&v[i];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float f = bf2f(hv[q]);
        if (mode == POOL_AVG) {
          sum[q] += f;
        } else {
          const float key = mode == POOL_MAXABS ? fabsf(f) : f;
          const float bk = mode == POOL_MAXABS ? fabsf(best[q]) : best[q];
          if (bi[q] < 0 || key > bk) { best[q] = f; bi[q] = i; }
        }
      }
    }
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      o[q] = f2bf(mode == POOL_AVG ? sum[q] / (float)max(cnt, 1) : best[q]);
    const long long yo = (long long)pix * C + cvu * 8;
    *(uint4*)(y + yo) = *(const uint4*)o;
    if (argmax && mode != POOL_AVG) {
      int a[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        int o2 = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) o2 = bi[q] == i ? off[i] : o2;
        a[q] = bi[q] < 0 ? -1 : (int)(img + o2) + q;
      }
      *(int4*)(argmax + yo) = make_int4(a[0], a[1], a[2], a[3]);
      *(int4*)(argmax + yo + 4) = make_int4(a[4], a[5], a[6], a[7]);
    }
  }
}

// gather backward: dx[n][h][w][c] = sum over windows covering (h,w)
template <int VEC, int MODE>
__global__ void pool_bwd_kernel(const uint16_t* dy, const int* argmax,
                                uint16_t* dx, int N, int H, int W, int C,
                                int OH, int OW, int ky, int kx, int sy, int sx,
                                int pt, int pl, int, const uint16_t* aux,
                                int aux_act, FastDiv fCV, FastDiv fW,
                                FastDiv fH, FastDiv fSy, FastDiv fSx) {
  const int CV = C / VEC;
  const int total = N * H * W * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, wu, nu, hu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fW, t, wu);
    fdivmod(t, fH, nu, hu);
    const int cv = cvu, w = wu, n = nu, h = hu;
    int xoff = pix * C + cv * VEC;
    // windows oh with oh*sy - pt <= h < oh*sy - pt + ky
    int hp = h + pt, wp = w + pl;
    int oh0 = hp - ky + 1 <= 0 ? 0 : (int)fdiv(hp - ky + sy, fSy);
    int oh1 = min(OH - 1, (int)fdiv(hp, fSy));
    int ow0 = wp - kx + 1 <= 0 ? 0 : (int)fdiv(wp - kx + sx, fSx);
    int ow1 = min(OW - 1, (int)fdiv(wp, fSx));
    float acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        int yo = ((n * OH + oh) * OW + ow) * C + cv * VEC;
        uint16_t g[VEC];
        if (VEC == 8) *(uint4*)g = *(const uint4*)(dy + yo);
        else if (VEC > 1) __builtin_memcpy(g, dy + yo, VEC * 2);
        else g[0] = dy[yo];
        if (MODE == POOL_AVG) {
          int hh0 = max(oh * sy - pt, 0), hh1 = min(oh * sy - pt + ky, H);
          int ww0 = max(ow * sx - pl, 0), ww1 = min(ow * sx - pl + kx, W);
          float inv = 1.f / (float)max((hh1 - hh0) * (ww1 - ww0), 1);
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[q] += bf2f(g[q]) * inv;
        } else {
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            if (argmax[yo + q] == xoff + q) acc[q] += bf2f(g[q]);
        }
      }
    uint16_t o[VEC];
    if (aux) {
      uint16_t a[VEC];
      if (VEC == 8) *(uint4*)a = *(const uint4*)(aux + xoff);
      else if (VEC > 1) __builtin_memcpy(a, aux + xoff, VEC * 2);
      else a[0] = aux[xoff];
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[q] *= act_bwd(bf2f(a[q]), aux_act);
    }
#pragma unroll
    for (int q = 0; q < VEC; ++q) o[q] = f2bf(acc[q]);
    if (VEC == 8) *(uint4*)(dx + xoff) = *(uint4*)o;
    else if (VEC > 1) __builtin_memcpy(dx + xoff, o, VEC * 2);
    else dx[xoff] = o[0];
  }
}


// 3x3 windows with stride >= 2: an input pixel lies in at most 2x2 windows;
// their dy / argmax loads are issued together (clamped addresses + masks).
template <int MODE>
__global__ void pool_bwd3_kernel(const uint16_t* __restrict__ dy,
                                 const int* __restrict__ argmax,
                                 uint16_t* __restrict__ dx, int N, int H,
                                 int W, int C, int OH, int OW, int sy, int sx,
                                 int pt, int pl, const uint16_t* aux,
                                 int aux_act, FastDiv fCV, FastDiv fW,
                                 FastDiv fH, FastDiv fSy, FastDiv fSx) {
  const int CV = C >> 3;
  const int total = N * H * W * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, wu, nu, hu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fW, t, wu);
    fdivmod(t, fH, nu, hu);
    const int xoff = (int)pix * C + (int)cvu * 8;
    const int hp = (int)hu + pt, wp = (int)wu + pl;
    // last window starting at or before hp; the one before it may also cover
    const int oh1 = min(OH - 1, (int)fdiv(hp, fSy));
    const int ow1 = min(OW - 1, (int)fdiv(wp, fSx));
    int yo[4];
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = oh1 - (i >> 1), ow = ow1 - (i & 1);
      ok[i] = oh >= 0 && ow >= 0 && hp - oh * sy < 3 && wp - ow * sx < 3 &&
              hp >= oh * sy && wp >= ow * sx;
      const int ohc = max(oh, 0), owc = max(ow, 0);
      yo[i] = (((int)nu * OH + ohc) * OW + owc) * C + (int)cvu * 8;
    }
    uint4 g[4];
    int4 a0[4], a1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      g[i] = *(const uint4*)(dy + yo[i]);
      if (MODE != POOL_AVG) {
        a0[i] = *(const int4*)(argmax + yo[i]);
        a1[i] = *(const int4*)(argmax + yo[i] + 4);
      }
    }
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!ok[i]) continue;
      const uint16_t* gv = (const uint16_t*)&g[i];
      if (MODE == POOL_AVG) {
        const int oh = oh1 - (i >> 1), ow = ow1 - (i & 1);
        const int hh0 = max(oh * sy - pt, 0), hh1 = min(oh * sy - pt + 3, H);
        const int ww0 = max(ow * sx - pl, 0), ww1 = min(ow * sx - pl + 3, W);
        const float inv = 1.f / (float)max((hh1 - hh0) * (ww1 - ww0), 1);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += bf2f(gv[q]) * inv;
      } else {
        const int am[8] = {a0[i].x, a0[i].y, a0[i].z, a0[i].w,
                           a1[i].x, a1[i].y, a1[i].z, a1[i].w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
          acc[q] += am[q] == xoff + q ? bf2f(gv[q]) : 0.f;
      }
    }
    if (aux) {
      float a[8];
      const uint4 av = *(const uint4*)(aux + xoff);
      const uint16_t* ah = (const uint16_t*)&av;
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = bf2f(ah[q]);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] *= act_bwd(a[q], aux_act);
    }
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(acc[q]);
    *(uint4*)(dx + xoff) = *(const uint4*)o;
  }
}

// 3x3 / stride-2 (unpadded) max pooling backward over 2x2 input blocks, the
// layout of lrn_pool3s2_bwd_dpp_kernel: a pixel of block (bh, bw) lies only
// in windows (bh - 1 + a, bw - 1 + b), so one thread loads those (at most)
// four windows' gradient + argmax once for its four pixels - the per-pixel
// kernel above loads them once per pixel, 3.25x the bytes through L2
// (AlexNet pool5: 13x13 -> 6x6).  An absent window's gradient is zeroed (its
// clamped twin's argmax may name one of these pixels).
template <int MODE>
__global__ __launch_bounds__(256) void pool_bwd3s2_blk_kernel(
    const uint16_t* __restrict__ dy, const int* __restrict__ argmax,
    uint16_t* __restrict__ dx, int N, int H, int W, int C, int OH, int OW,
    const uint16_t* aux, int aux_act, FastDiv fCV, FastDiv fBW,
    FastDiv fBH) {
  static_assert(MODE != POOL_AVG, "argmax-based modes");
  const int CV = C >> 3;
  const int BH = (H + 1) >> 1, BW = (W + 1) >> 1;
  const uint32_t total = (uint32_t)N * BH * BW * CV;
  const uint32_t OWC = (uint32_t)OW * C;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t blk, cvu, t, bwu, nu, bhu;
    fdivmod(e, fCV, blk, cvu);
    fdivmod(blk, fBW, t, bwu);
    fdivmod(t, fBH, nu, bhu);
    const uint32_t c0 = cvu * 8;
    const uint32_t orow[2] = {(bhu > 0 ? bhu - 1 : 0), min(bhu, (uint32_t)OH - 1)};
    const uint32_t ocol[2] = {(bwu > 0 ? bwu - 1 : 0), min(bwu, (uint32_t)OW - 1)};
    const bool rok[2] = {bhu > 0, bhu < (uint32_t)OH};
    const bool cok[2] = {bwu > 0, bwu < (uint32_t)OW};
    uint4 g[4];
    int4 a0[4], a1[4];
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const int a = wi >> 1, b = wi & 1;
      const uint32_t yo =
          (nu * OH + orow[a]) * OWC + ocol[b] * (uint32_t)C + c0;
      const uint4 gv = *(const uint4*)(dy + yo);
      g[wi] = rok[a] && cok[b] ? gv : make_uint4(0u, 0u, 0u, 0u);
      a0[wi] = *(const int4*)(argmax + yo);
      a1[wi] = *(const int4*)(argmax + yo + 4);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t hp = 2 * bhu + (p >> 1), wp = 2 * bwu + (p & 1);
      const bool pv = hp < (uint32_t)H && wp < (uint32_t)W;
      const uint32_t xoff = ((nu * H + hp) * W + wp) * C + c0;
      float acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll
      for (int wi = 0; wi < 4; ++wi) {
        const int a = wi >> 1, b = wi & 1;
        // window-local row / column of pixel p in window (bh-1+a, bw-1+b)
        const int r = 2 * (1 - a) + (p >> 1), c = 2 * (1 - b) + (p & 1);
        if (r > 2 || c > 2) continue;
        const uint16_t* gv = (const uint16_t*)&g[wi];
        const int am[8] = {a0[wi].x, a0[wi].y, a0[wi].z, a0[wi].w,
                           a1[wi].x, a1[wi].y, a1[wi].z, a1[wi].w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
          acc[q] += am[q] == (int)xoff + q ? bf2f(gv[q]) : 0.f;
      }
      if (aux) {
        const uint4 av4 = *(const uint4*)(aux + (pv ? xoff : c0));
        const uint16_t* ah = (const uint16_t*)&av4;
        float av[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) av[q] = bf2f(ah[q]);
        act_bwd_mul8(acc, av, aux_act);
      }
      if (pv) *(uint4*)(dx + xoff) = pack_bf16x8(acc);
    }
  }
}

// backward selector for A/B runs (hvk_set_pool_bwd_variant): 0 the 2x2-block
// kernel for unpadded 3x3 / stride-2 max pooling, 1 the per-pixel kernel
static int g_pool_bwd_variant = 0;
HVK_API void hvk_set_pool_bwd_variant(int v) { g_pool_bwd_variant = v; }

// LRN across channels: s_c = k + alpha * sum_{|c'-c|<=n/2} x_c'^2 ;
// y_c = x_c * s_c^-beta.  One wave per pixel; channels staged in LDS.
constexpr int LRN_MAXC = 1024;
__global__ void lrn_fwd_kernel(const uint16_t* x, uint16_t* y, long long P,
                               int C, int n, float alpha, float beta, float k) {
  __shared__ float sx[4][LRN_MAXC];
  int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* xs = sx[wv];
  int half = n / 2;
  for (long long p = (long long)blockIdx.x * 4 + wv; p < P;
       p += (long long)gridDim.x * 4) {
    const uint16_t* xp = x + p * C;
    for (int c = lane; c < C; c += 64) xs[c] = bf2f(xp[c]);
    __builtin_amdgcn_wave_barrier();
    for (int c = lane; c < C; c += 64) {
      float s = 0.f;
      int c0 = max(0, c - half), c1 = min(C - 1, c + half);
      for (int j = c0; j <= c1; ++j) s += xs[j] * xs[j];
      s = k + alpha * s;
      y[p * C + c] = f2bf(xs[c] * ex2(-beta * log2f(s)));
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void lrn_bwd_kernel(const uint16_t* x, const uint16_t* dy,
                               uint16_t* dx, long long P, int C, int n,
                               float alpha, float beta, float k,
                               const uint16_t* aux, int aux_act) {
  __shared__ float sx[4][LRN_MAXC];
  __shared__ float st[4][LRN_MAXC];
  int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* xs = sx[wv];
  float* ts = st[wv];
  int half = n / 2;
  for (long long p = (long long)blockIdx.x * 4 + wv; p < P;
       p += (long long)gridDim.x * 4) {
    for (int c = lane; c < C; c += 64) xs[c] = bf2f(x[p * C + c]);
    __builtin_amdgcn_wave_barrier();
    // t_c = dy_c * x_c * s_c^(-beta-1); keep s_c^-beta * dy_c in registers
    float keep[LRN_MAXC / 64];
#pragma unroll
    for (int idx = 0; idx < LRN_MAXC / 64; ++idx) {
      int c = lane + idx * 64;
      if (c >= C) break;
      float s = 0.f;
      int c0 = max(0, c - half), c1 = min(C - 1, c + half);
      for (int j = c0; j <= c1; ++j) s += xs[j] * xs[j];
      s = k + alpha * s;
      float sb = ex2(-beta * log2f(s));
      float g = bf2f(dy[p * C + c]);
      ts[c] = g * xs[c] * sb / s;
      keep[idx] = g * sb;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int idx = 0; idx < LRN_MAXC / 64; ++idx) {
      int c = lane + idx * 64;
      if (c >= C) break;
      float acc = 0.f;
      int c0 = max(0, c - half), c1 = min(C - 1, c + half);
      for (int j = c0; j <= c1; ++j) acc += ts[j];
      float v = keep[idx] - 2.f * alpha * beta * xs[c] * acc;
      if (aux) v *= act_bwd(bf2f(aux[p * C + c]), aux_act);
      dx[p * C + c] = f2bf(v);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Vectorised LRN (C % 8 == 0, n/2 <= 4): a thread owns 8 channels of one
// pixel and reads the neighbouring 8-channel chunks for the window halo;
// all arrays are compile-time indexed (registers, no scratch).
__device__ __forceinline__ void load8(const uint16_t* p, float* d) {
  uint4 v = *(const uint4*)p;
  const uint16_t* h = (const uint16_t*)&v;
#pragma unroll
  for (int q = 0; q < 8; ++q) d[q] = bf2f(h[q]);
}
__device__ __forceinline__ void load24(const uint16_t* row, int c0, int C,
                                       float* d) {
#pragma unroll
  for (int q = 0; q < 24; ++q) d[q] = 0.f;
  if (c0 >= 8) load8(row + c0 - 8, d);
  load8(row + c0, d + 8);
  if (c0 + 8 < C) load8(row + c0 + 8, d + 16);
}
__device__ __forceinline__ void load4(const uint16_t* p, float* d) {
  const uint2 v = *(const uint2*)p;
  d[0] = __uint_as_float(v.x << 16);
  d[1] = __uint_as_float(v.x & 0xffff0000u);
  d[2] = __uint_as_float(v.y << 16);
  d[3] = __uint_as_float(v.y & 0xffff0000u);
}
// d[k] = row[c0 - 8 + k] for the channels an LRN of half-width `half` over
// channels [c0 - half, c0 + 8 + half) reads (zero outside [0, C)): 16
// channels (8 B + 16 B + 8 B) when half <= 2, else the full 24.
template <int half>
__device__ __forceinline__ void loadx(const uint16_t* row, int c0, int C,
                                      float* d) {
  if (half > 2) {
    load24(row, c0, C, d);
    return;
  }
#pragma unroll
  for (int q = 0; q < 24; ++q) d[q] = 0.f;
  if (c0 >= 8) load4(row + c0 - 4, d + 4);
  load8(row + c0, d + 8);
  if (c0 + 8 < C) load4(row + c0 + 8, d + 16);
}
template <int half>
__global__ void lrn_fwd_vec_kernel(const uint16_t* x, uint16_t* y, int P,
                                   int C, float alpha, float beta,
                                   float k, FastDiv fCV) {
  const int CV = C >> 3;
  const int total = P * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    int p = (int)fdiv((uint32_t)e, fCV);
    int c0 = (e - p * CV) << 3;
    const uint16_t* row = x + (long long)p * C;
    float v[24];
    load24(row, c0, C, v);
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float s = 0.f;
#pragma unroll
      for (int d = -4; d <= 4; ++d) {
        float t = v[8 + q + d];
        s += (d >= -half && d <= half) ? t * t : 0.f;
      }
      s = k + alpha * s;
      o[q] = f2bf(v[8 + q] * ex2(-beta * __log2f(s)));
    }
    *(uint4*)(y + (long long)p * C + c0) = *(uint4*)o;
  }
}
template <int half>
__global__ void lrn_bwd_vec_kernel(const uint16_t* x, const uint16_t* dy,
                                   uint16_t* dx, int P, int C,
                                   float alpha, float beta, float k,
                                   const uint16_t* aux, int aux_act,
                                   FastDiv fCV) {
  const int CV = C >> 3;
  const int total = P * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    int p = (int)fdiv((uint32_t)e, fCV);
    int c0 = (e - p * CV) << 3;
    long long base = (long long)p * C;
    float xv[24], gv[24];
    load24(x + base, c0, C, xv);
    load24(dy + base, c0, C, gv);
    // t_j = dy_j x_j s_j^(-beta-1) for j in [c0-4, c0+12) (16 values)
    float tj[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = -4; d <= 4; ++d) {
        int idx = 4 + j + d;
        float t = (idx >= 0 && idx < 24) ? xv[idx] : 0.f;
        s += (d >= -half && d <= half) ? t * t : 0.f;
      }
      s = k + alpha * s;
      const float ls = __log2f(s);
      float sb = ex2(-beta * ls);
      // s^(-beta-1) as a second exp instead of a division
      tj[j] = gv[4 + j] * xv[4 + j] * ex2((-beta - 1.f) * ls);
      // keep s^-beta of the owned channels in gv's free slots? recompute
      // below instead (cheap)
      if (j >= 4 && j < 12) xv[(j - 4) + 0] = sb;  // xv[0..7] unused now
    }
    uint16_t o[8];
    float a[8];
    if (aux) load8(aux + base + c0, a);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float acc = 0.f;
#pragma unroll
      for (int d = -4; d <= 4; ++d)
        acc += (d >= -half && d <= half) ? tj[4 + q + d] : 0.f;
      float v = gv[8 + q] * xv[q] - 2.f * alpha * beta * xv[8 + q] * acc;
      if (aux) v *= act_bwd(a[q], aux_act);
      o[q] = f2bf(v);
    }
    *(uint4*)(dx + base + c0) = *(uint4*)o;
  }
}

// ---------------------------------------------------------------------------
// LRN -> 3x3 max pooling fused (AlexNet norm1/pool1, norm2/pool2): the LRN
// output is never written.  Forward: per pool output x 8 channels, the LRN
// of the 9 window pixels is recomputed from x (24-channel halo loads) and
// max-pooled; argmax is the offset into the (virtual) LRN output, i.e. the
// same tensor geometry as x.  Backward: per input pixel x 8 channels, the
// pool gradient of the 16 channels the LRN window needs is gathered from
// the <= 2 x 2 covering windows, then the LRN backward of lrn_bwd_vec runs
// on it - the pool-gradient tensor is never written either.
__device__ __forceinline__ float lrn_s(const float* v, int c, int half,
                                      float alpha, float k) {
  float s = 0.f;
#pragma unroll
  for (int d = -4; d <= 4; ++d) {
    const int idx = c + d;
    const float t = (idx >= 0 && idx < 24) ? v[idx] : 0.f;
    s += (d >= -half && d <= half) ? t * t : 0.f;
  }
  return k + alpha * s;
}

template <int half>
__global__ void lrn_pool3_fwd_kernel(const uint16_t* __restrict__ x,
                                     uint16_t* __restrict__ y,
                                     int* __restrict__ argmax, int N, int H,
                                     int W, int C, int OH, int OW, int sy,
                                     int sx, float alpha, float beta, float k,
                                     FastDiv fCV, FastDiv fOW, FastDiv fOH) {
  const int CV = C >> 3;
  const int total = N * OH * OW * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const int c0 = (int)cvu * 8;
    const int h0 = (int)ohu * sy, w0 = (int)owu * sx;
    const long long img = (long long)nu * H * W * C;
    float best[8];
    int bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { best[q] = -INFINITY; bi[q] = -1; }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int h = h0 + i / 3, w = w0 + i % 3;
      if (h >= H || w >= W) continue;
      const int off = (h * W + w) * C;
      float v[24];
      loadx<half>(x + img + off, c0, C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float s = lrn_s(v, 8 + q, half, alpha, k);
        const float yv = v[8 + q] * ex2(-beta * __log2f(s));
        if (bi[q] < 0 || yv > best[q]) { best[q] = yv; bi[q] = off; }
      }
    }
    uint16_t o[8];
    int a[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = f2bf(best[q]);
      a[q] = (int)(img + bi[q]) + c0 + q;
    }
    const long long yo = (long long)pix * C + c0;
    *(uint4*)(y + yo) = *(const uint4*)o;
    *(int4*)(argmax + yo) = make_int4(a[0], a[1], a[2], a[3]);
    *(int4*)(argmax + yo + 4) = make_int4(a[4], a[5], a[6], a[7]);
  }
}

template <int half>
__global__ void lrn_pool3_bwd_kernel(const uint16_t* __restrict__ x,
                                     const uint16_t* __restrict__ dp,
                                     const int* __restrict__ argmax,
                                     uint16_t* __restrict__ dx, int N, int H,
                                     int W, int C, int OH, int OW, int sy,
                                     int sx, float alpha, float beta, float k,
                                     const uint16_t* aux, int aux_act,
                                     FastDiv fCV, FastDiv fW, FastDiv fH,
                                     FastDiv fSy, FastDiv fSx) {
  const int CV = C >> 3;
  const int total = N * H * W * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, wu, nu, hu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fW, t, wu);
    fdivmod(t, fH, nu, hu);
    const int c0 = (int)cvu * 8;
    const long long base = (long long)pix * C;
    // covering windows (3x3, stride >= 2): at most 2 x 2
    const int oh1 = min(OH - 1, (int)fdiv(hu, fSy));
    const int ow1 = min(OW - 1, (int)fdiv(wu, fSx));
    int yo[4];
    bool ok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = oh1 - (i >> 1), ow = ow1 - (i & 1);
      ok[i] = oh >= 0 && ow >= 0 && (int)hu - oh * sy < 3 &&
              (int)wu - ow * sx < 3 && (int)hu >= oh * sy &&
              (int)wu >= ow * sx;
      yo[i] = (((int)nu * OH + max(oh, 0)) * OW + max(ow, 0)) * C;
    }
    // g[j] = pool gradient at channel c0 - 8 + j (j < 24), zero outside C
    float g[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) g[j] = 0.f;
#pragma unroll
    for (int part = 0; part < 3; ++part) {
      const int cb = c0 - 8 + part * 8;
      if (cb < 0 || cb >= C) continue;
      const int xo = (int)base + cb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!ok[i]) continue;
        const uint4 gv = *(const uint4*)(dp + yo[i] + cb);
        const int4 a0 = *(const int4*)(argmax + yo[i] + cb);
        const int4 a1 = *(const int4*)(argmax + yo[i] + cb + 4);
        const uint16_t* gh = (const uint16_t*)&gv;
        const int am[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
          g[part * 8 + q] += am[q] == xo + q ? bf2f(gh[q]) : 0.f;
      }
    }
    float xv[24];
    loadx<half>(x + base, c0, C, xv);
    // t_j = g_j x_j s_j^(-beta-1), j in [c0-4, c0+12)
    float tj[16], sb[8];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float s = lrn_s(xv, 4 + j, half, alpha, k);
      const float ls = __log2f(s);
      tj[j] = g[4 + j] * xv[4 + j] * ex2((-beta - 1.f) * ls);
      if (j >= 4 && j < 12) sb[j - 4] = ex2(-beta * ls);
    }
    float a[8];
    if (aux) load8(aux + base + c0, a);
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float acc = 0.f;
#pragma unroll
      for (int d = -4; d <= 4; ++d)
        acc += (d >= -half && d <= half) ? tj[4 + q + d] : 0.f;
      float v = g[8 + q] * sb[q] - 2.f * alpha * beta * xv[8 + q] * acc;
      if (aux) v *= act_bwd(a[q], aux_act);
      o[q] = f2bf(v);
    }
    *(uint4*)(dx + base + c0) = *(const uint4*)o;
  }
}

// Stride-2 specialisation of lrn_pool3_bwd_kernel: one thread per 2 x 2 input
// pixel block x 8 channels.  With 3x3 / stride 2 windows the four windows
// (i-1..i) x (j-1..j) cover the whole block (i, j), so each (window, 4-channel
// chunk) of pool gradient + argmax is loaded once per block instead of once
// per covering pixel and 8-channel part (~6x fewer vector-memory bytes; the
// old kernel was texture-address bound, not HBM bound).  When aux is x itself
// (ReLU below, derivative from the output) the activation derivative reuses
// the x registers.
template <int half>
__global__ __launch_bounds__(256) void lrn_pool3s2_bwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dp,
    const int* __restrict__ argmax, uint16_t* __restrict__ dx, int N, int H,
    int W, int C, int OH, int OW, float alpha, float beta, float k,
    const uint16_t* aux, int aux_act, FastDiv fCV, FastDiv fBW,
    FastDiv fBH) {
  const int CV = C >> 3;
  const int BH = (H + 1) >> 1, BW = (W + 1) >> 1;
  const int total = N * BH * BW * CV;
  const bool aux_x = aux == x;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t blk, cvu, t, bwu, nu, bhu;
    fdivmod((uint32_t)e, fCV, blk, cvu);
    fdivmod(blk, fBW, t, bwu);
    fdivmod(t, fBH, nu, bhu);
    const int c0 = (int)cvu * 8;
    int po[4];
    bool pv[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int hp = (int)bhu * 2 + (p >> 1), wp = (int)bwu * 2 + (p & 1);
      pv[p] = hp < H && wp < W;
      // argmax values are >= 0: an invalid pixel never matches
      po[p] = pv[p] ? (((int)nu * H + hp) * W + wp) * C : -1;
    }
    // g[p][j]: pool gradient of pixel p at channel c0 - 4 + j
    float g[4][16];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < 16; ++j) g[p][j] = 0.f;
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const int oh = (int)bhu - 1 + (wi >> 1), ow = (int)bwu - 1 + (wi & 1);
      if (oh < 0 || ow < 0 || oh >= OH || ow >= OW) continue;
      const int yo = (((int)nu * OH + oh) * OW + ow) * C;
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const int cb = c0 - 4 + ch * 4;
        if (cb < 0 || cb >= C) continue;
        float gf[4];
        load4(dp + yo + cb, gf);
        const int4 a4 = *(const int4*)(argmax + yo + cb);
        const int am[4] = {a4.x - cb, a4.y - cb - 1, a4.z - cb - 2,
                           a4.w - cb - 3};
        // window (i-1+a, j-1+b) reaches pixel (ph, pw) of the block only if
        // (a || !ph) && (b || !pw): 9 of the 16 (window, pixel) pairs
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          if (!((wi >> 1) || !(p >> 1)) || !((wi & 1) || !(p & 1))) continue;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            g[p][ch * 4 + q] += am[q] == po[p] ? gf[q] : 0.f;
        }
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (!pv[p]) continue;
      float xv[24];
      loadx<half>(x + po[p], c0, C, xv);
      float tj[16], sb[8];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float s = lrn_s(xv, 4 + j, half, alpha, k);
        const float ls = __log2f(s);
        const float e1 = ex2((-beta - 1.f) * ls);  // s^(-beta-1)
        tj[j] = g[p][j] * xv[4 + j] * e1;
        if (j >= 4 && j < 12) sb[j - 4] = e1 * s;  // s^-beta
      }
      float a[8];
      if (aux && !aux_x) load8(aux + po[p] + c0, a);
      uint16_t o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float acc = 0.f;
#pragma unroll
        for (int d = -4; d <= 4; ++d)
          acc += (d >= -half && d <= half) ? tj[4 + q + d] : 0.f;
        float v = g[p][4 + q] * sb[q] - 2.f * alpha * beta * xv[8 + q] * acc;
        if (aux) v *= act_bwd(aux_x ? xv[8 + q] : a[q], aux_act);
        o[q] = f2bf(v);
      }
      *(uint4*)(dx + po[p] + c0) = *(const uint4*)o;
    }
  }
}
// ---------------------------------------------------------------------------
// Non-overlapping 2 x 2 / stride-2 pooling (VGG) WITHOUT an argmax tensor.
// Forward: one thread per output pixel x 8 channels, four 16-B loads, one
// 16-B store.  Backward recomputes the window's choice from the forward input
// (the first maximum in window order, as the forward took it) and writes all
// four input pixels of the window: it reads x + dy instead of dy + an int32
// argmax as large as x / 2, and the forward writes no argmax at all.  Even H
// and W only (every input pixel belongs to exactly one window).
// q8.q (optional): also the fp8 copy of y for the next fp8 layer (fused
// quantisation, fp8_common.h)
template <int MODE>
__global__ __launch_bounds__(256) void pool2_fwd_kernel(
    const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int N, int H,
    int W, int C, FastDiv fCV, FastDiv fOW, FastDiv fOH, Q8 q8) {
  const int CV = C >> 3, OH = H >> 1, OW = W >> 1;
  const int total = N * OH * OW * CV;
  const float qs = q8.q ? fp8_scale(q8.st, q8.hist, q8.fmax) : 1.f;
  float amax = 0.f;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const long long b = (((long long)nu * H + 2 * ohu) * W + 2 * owu) * C +
                        cvu * 8;
    uint4 v[4];
    v[0] = *(const uint4*)(x + b);
    v[1] = *(const uint4*)(x + b + C);
    v[2] = *(const uint4*)(x + b + (long long)W * C);
    v[3] = *(const uint4*)(x + b + (long long)W * C + C);
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float best = 0.f, key = -INFINITY, sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float f = bf2f(((const uint16_t*)&v[i])[q]);
        sum += f;
        const float kf = MODE == POOL_MAXABS ? fabsf(f) : f;
        if (i == 0 || kf > key) { key = kf; best = f; }
      }
      o[q] = f2bf(MODE == POOL_AVG ? 0.25f * sum : best);
    }
    const long long yo = (long long)pix * C + cvu * 8;
    *(uint4*)(y + yo) = *(const uint4*)o;
    if (q8.q) q8_store8(q8, yo, *(const uint4*)o, qs, amax);
  }
  if (q8.q) {
    __shared__ float red[4];
    q8_block_amax(q8, amax, red);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void pool2_bwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
    uint16_t* __restrict__ dx, int N, int H, int W, int C,
    const uint16_t* aux, int aux_act, FastDiv fCV, FastDiv fOW,
    FastDiv fOH, Q8 q8) {
  const int CV = C >> 3, OH = H >> 1, OW = W >> 1;
  const int total = N * OH * OW * CV;
  const float qs = q8.q ? fp8_scale(q8.st, q8.hist, q8.fmax) : 1.f;
  float amax = 0.f;
  const bool aux_x = aux == x;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const long long b = (((long long)nu * H + 2 * ohu) * W + 2 * owu) * C +
                        cvu * 8;
    const long long off[4] = {b, b + C, b + (long long)W * C,
                              b + (long long)W * C + C};
    const uint4 g = *(const uint4*)(dy + (long long)pix * C + cvu * 8);
    uint4 v[4], a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (MODE != POOL_AVG || aux_x) v[i] = *(const uint4*)(x + off[i]);
      if (aux && !aux_x) a[i] = *(const uint4*)(aux + off[i]);
    }
    uint16_t o[4][8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float gq = bf2f(((const uint16_t*)&g)[q]);
      int ch = 0;
      if (MODE != POOL_AVG) {
        float key = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float f = bf2f(((const uint16_t*)&v[i])[q]);
          const float kf = MODE == POOL_MAXABS ? fabsf(f) : f;
          if (i == 0 || kf > key) { key = kf; ch = i; }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float d = MODE == POOL_AVG ? 0.25f * gq : (i == ch ? gq : 0.f);
        if (aux) {
          const float av = bf2f(((const uint16_t*)(aux_x ? &v[i] : &a[i]))[q]);
          d *= act_bwd(av, aux_act);
        }
        o[i][q] = f2bf(d);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *(uint4*)(dx + off[i]) = *(const uint4*)o[i];
      if (q8.q) q8_store8(q8, off[i], *(const uint4*)o[i], qs, amax);
    }
  }
  if (q8.q) {
    __shared__ float red[4];
    q8_block_amax(q8, amax, red);
  }
}

// ---------------------------------------------------------------------------
// Fused LRN -> 3x3 / stride-2 max pooling with a ONE-BYTE argmax: the index
// (0..8, row-major) of the chosen pixel inside its window instead of an int32
// offset into x.  Forward writes 8 B of argmax per 8 channels instead of 32 B;
// backward reads one 8-B chunk per 8 channels and compares it against the
// window-local index a block pixel has in each of its 2 x 2 covering windows
// (a compile-time constant per (window, pixel) pair).  The LRN loops only
// evaluate the channels the window half-width needs.
template <int half>
__global__ __launch_bounds__(256) void lrn_pool3s2_fwd_u8_kernel(
    const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
    uint8_t* __restrict__ argmax, int N, int H, int W, int C, int OH, int OW,
    float alpha, float beta, float k, FastDiv fCV, FastDiv fOW, FastDiv fOH) {
  const int CV = C >> 3;
  const int total = N * OH * OW * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const int c0 = (int)cvu * 8;
    const int h0 = (int)ohu * 2, w0 = (int)owu * 2;
    const uint16_t* img = x + (long long)nu * H * W * C;
    float best[8];
    int bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) { best[q] = -INFINITY; bi[q] = 0; }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int h = h0 + i / 3, w = w0 + i % 3;
      if (h >= H || w >= W) continue;
      float v[24];
      loadx<half>(img + (h * W + w) * C, c0, C, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float s = lrn_s(v, 8 + q, half, alpha, k);
        const float yv = v[8 + q] * ex2(-beta * __log2f(s));
        if (i == 0 || yv > best[q]) { best[q] = yv; bi[q] = i; }
      }
    }
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(best[q]);
    const long long yo = (long long)pix * C + c0;
    *(uint4*)(y + yo) = *(const uint4*)o;
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(argmax + yo) = a;
  }
}

// The same forward (half <= 2) with every window pixel's 16 channels
// loaded before any arithmetic: the 9 x 32-B loads of a thread are all in
// flight at once (clamped in-range addresses, out-of-window taps masked
// afterwards) instead of one pixel's loads per LRN evaluation - the kernel
// is bound by memory latency, not by its transcendental work (a 2 x 2
// outputs-per-thread variant that evaluated 31 % fewer LRN pixels ran at the
// same speed: profiles/r3_experiments.md).  Same arithmetic and window order:
// bit-identical to lrn_pool3s2_fwd_u8_kernel.
template <int half>
__global__ __launch_bounds__(256) void lrn_pool3s2_fwd_u8p_kernel(
    const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
    uint8_t* __restrict__ argmax, int N, int H, int W, int C, int OH, int OW,
    float alpha, float beta, float k, FastDiv fCV, FastDiv fOW, FastDiv fOH) {
  static_assert(half <= 2, "16-channel halo");
  const int CV = C >> 3;
  const int total = N * OH * OW * CV;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t pix, cvu, t, owu, nu, ohu;
    fdivmod((uint32_t)e, fCV, pix, cvu);
    fdivmod(pix, fOW, t, owu);
    fdivmod(t, fOH, nu, ohu);
    const int c0 = (int)cvu * 8;
    const int h0 = (int)ohu * 2, w0 = (int)owu * 2;
    const uint16_t* img = x + (long long)nu * H * W * C;
    const int clo = c0 >= 8 ? c0 - 4 : c0;        // in-range halo addresses
    const int chi = c0 + 8 < C ? c0 + 8 : c0 + 4;
    uint2 lo[9], hi[9];
    uint4 mid[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int h = min(h0 + i / 3, H - 1), w = min(w0 + i % 3, W - 1);
      const uint16_t* row = img + ((long long)h * W + w) * C;
      lo[i] = *(const uint2*)(row + clo);
      mid[i] = *(const uint4*)(row + c0);
      hi[i] = *(const uint2*)(row + chi);
    }
    float best[8];
    int bi[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const bool in = h0 + i / 3 < H && w0 + i % 3 < W;
      float v[24];
#pragma unroll
      for (int q = 0; q < 24; ++q) v[q] = 0.f;
      if (c0 >= 8) {
        v[4] = __uint_as_float(lo[i].x << 16);
        v[5] = __uint_as_float(lo[i].x & 0xffff0000u);
        v[6] = __uint_as_float(lo[i].y << 16);
        v[7] = __uint_as_float(lo[i].y & 0xffff0000u);
      }
      const uint32_t m[4] = {mid[i].x, mid[i].y, mid[i].z, mid[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[8 + 2 * q] = __uint_as_float(m[q] << 16);
        v[9 + 2 * q] = __uint_as_float(m[q] & 0xffff0000u);
      }
      if (c0 + 8 < C) {
        v[16] = __uint_as_float(hi[i].x << 16);
        v[17] = __uint_as_float(hi[i].x & 0xffff0000u);
        v[18] = __uint_as_float(hi[i].y << 16);
        v[19] = __uint_as_float(hi[i].y & 0xffff0000u);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float sv = lrn_s(v, 8 + q, half, alpha, k);
        const float yv = v[8 + q] * ex2(-beta * __log2f(sv));
        if (i == 0 || (in && yv > best[q])) { best[q] = yv; bi[q] = i; }
      }
    }
    uint16_t o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(best[q]);
    const long long yo = (long long)pix * C + c0;
    *(uint4*)(y + yo) = *(const uint4*)o;
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(argmax + yo) = a;
  }
}

// The same forward as a vertical walk: a thread owns one output column
// (x 8 channels) over a strip of R output rows.  Consecutive windows share
// an input row (window oh covers rows 2oh .. 2oh+2), so after the strip's
// first window each output row evaluates the LRN of 6 window pixels instead
// of 9, and the column max of the shared row (value and column index) is
// carried into the next window.  The LRN runs on PAIRS of pixels (row
// 2oh+1 and row 2oh+2 of one column) in float2 lanes, so its squares, window
// sums, scale and product are v_pk_* instructions.  Per channel the
// arithmetic, its order and the window scan order are those of
// lrn_pool3s2_fwd_u8_kernel (first maximum in row-major window order): the
// outputs and argmax bytes are bit-identical.  half <= 2: the halo is the
// dword on each side of the thread's 8 channels.
typedef float f32x2v __attribute__((ext_vector_type(2)));

struct LrnPx {   // one pixel's channels c0-2 .. c0+9 (bf16 pairs)
  uint32_t lo, hi;
  uint4 mid;
};

__device__ __forceinline__ LrnPx lrn_ldpx(const uint16_t* px, int c0,
                                          bool has_lo, bool has_hi) {
  LrnPx r;
  // in-range addresses always (c0 for an absent halo), zeroed after
  const uint32_t lo = *(const uint32_t*)(px + (has_lo ? c0 - 2 : c0));
  const uint32_t hi = *(const uint32_t*)(px + (has_hi ? c0 + 8 : c0));
  r.mid = *(const uint4*)(px + c0);
  r.lo = has_lo ? lo : 0u;
  r.hi = has_hi ? hi : 0u;
  return r;
}

// y[q] = x * (k + alpha * sum of the window's squares)^-beta for channels
// c0 + q of pixel a (.x) and pixel b (.y)
template <int half>
__device__ __forceinline__ void lrn_pair(const LrnPx& a, const LrnPx& b,
                                         float alpha, float beta, float k,
                                         f32x2v* y) {
  f32x2v v[12];
  auto up = [](uint32_t ua, uint32_t ub, f32x2v& l, f32x2v& h) {
    l = f32x2v{__uint_as_float(ua << 16), __uint_as_float(ub << 16)};
    h = f32x2v{__uint_as_float(ua & 0xffff0000u),
               __uint_as_float(ub & 0xffff0000u)};
  };
  up(a.lo, b.lo, v[0], v[1]);
  up(a.mid.x, b.mid.x, v[2], v[3]);
  up(a.mid.y, b.mid.y, v[4], v[5]);
  up(a.mid.z, b.mid.z, v[6], v[7]);
  up(a.mid.w, b.mid.w, v[8], v[9]);
  up(a.hi, b.hi, v[10], v[11]);
  f32x2v e[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) e[j] = v[j] * v[j];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    // ascending channel order from 0, as lrn_s
    f32x2v w = e[q + 2 - half];
#pragma unroll
    for (int d = 1 - half; d <= half; ++d) w = w + e[q + 2 + d];
    const f32x2v sv = k + alpha * w;
    f32x2v l2 = f32x2v{__log2f(sv.x), __log2f(sv.y)};
    l2 = -beta * l2;
    y[q] = v[q + 2] * f32x2v{ex2(l2.x), ex2(l2.y)};
  }
}

// at most 128 VGPRs (4 waves per SIMD instead of 3 at the unconstrained
// 151; no scratch)
template <int half, bool PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
void lrn_pool3s2_fwd_walk_kernel(
    const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
    uint8_t* __restrict__ argmax, int N, int H, int W, int C, int OH, int OW,
    int R, int S, float alpha, float beta, float k, FastDiv fCV, FastDiv fOW,
    FastDiv fS) {
  static_assert(half >= 1 && half <= 2, "dword halo");
  const int CV = C >> 3;
  const int total = N * S * OW * CV;
  // 32-bit element offsets (the host checks N H W C < 2^31)
  const uint32_t WC = (uint32_t)W * C, HWC = (uint32_t)H * WC;
  const uint32_t lastrow = (uint32_t)(H - 1) * WC;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t t1, cvu, t2, owu, nu, su;
    fdivmod((uint32_t)e, fCV, t1, cvu);
    fdivmod(t1, fOW, t2, owu);
    fdivmod(t2, fS, nu, su);
    const int c0 = (int)cvu * 8, w0 = (int)owu * 2;
    const int oh0 = (int)su * R, oh1 = min(OH, oh0 + R);
    const bool has_lo = c0 >= 8, has_hi = c0 + 8 < C;
    const uint16_t* img = x + nu * HWC;
    // every window lies inside the image (the host passes OH = (H - 3) / 2
    // + 1, OW likewise): no edge masks (they held ~50 SGPRs, spilled to VGPR
    // lanes)
    const int wc1 = w0 + 1, wc2 = w0 + 2;
    const uint32_t col[3] = {(uint32_t)w0 * C, (uint32_t)wc1 * C,
                             (uint32_t)wc2 * C};
    // pixel (row offset ro, window column j)
    auto px = [&](uint32_t ro, int j) { return img + ro + col[j]; };
    // column max of a row: value and column (first maximum)
    auto rowmax = [&](float y0, float y1v, float y2v, float& b, int& bi) {
      b = y0;
      bi = 0;
      if (y1v > b) { b = y1v; bi = 1; }
      if (y2v > b) { b = y2v; bi = 2; }
    };
    float cb[8];
    int ci[8];
    {   // the strip's first window row
      const uint32_t ro = 2u * oh0 * WC;
      const LrnPx p0 = lrn_ldpx(px(ro, 0), c0, has_lo, has_hi);
      const LrnPx p1 = lrn_ldpx(px(ro, 1), c0, has_lo, has_hi);
      const LrnPx p2 = lrn_ldpx(px(ro, 2), c0, has_lo, has_hi);
      f32x2v ya[8], yb[8];
      lrn_pair<half>(p0, p1, alpha, beta, k, ya);
      lrn_pair<half>(p2, p2, alpha, beta, k, yb);
#pragma unroll
      for (int q = 0; q < 8; ++q) rowmax(ya[q].x, ya[q].y, yb[q].x, cb[q], ci[q]);
    }
    // rows 2oh+1 / 2oh+2 of the three window columns; the next output
    // row's six pixels are loaded before this row's arithmetic (clamped
    // row indexes: always in range, masked by r1v / r2v when used)
    LrnPx a[3], b[3];
    auto load_rows = [&](int oh, LrnPx* ra, LrnPx* rb) {
      const uint32_t r1 = (uint32_t)(2 * oh + 1) * WC;
      const uint32_t hc1 = min(r1, lastrow), hc2 = min(r1 + WC, lastrow);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        ra[j] = lrn_ldpx(px(hc1, j), c0, has_lo, has_hi);
        rb[j] = lrn_ldpx(px(hc2, j), c0, has_lo, has_hi);
      }
    };
    load_rows(oh0, a, b);
    for (int oh = oh0; oh < oh1; ++oh) {
      LrnPx na[3], nb[3];
      if constexpr (PF) load_rows(min(oh + 1, oh1 - 1), na, nb);
      else if (oh > oh0) load_rows(oh, a, b);
      f32x2v yc[3][8];
#pragma unroll
      for (int c = 0; c < 3; ++c) lrn_pair<half>(a[c], b[c], alpha, beta, k, yc[c]);
      uint16_t o[8];
      uint8_t ai[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float b1, b2;
        int i1, i2;
        rowmax(yc[0][q].x, yc[1][q].x, yc[2][q].x, b1, i1);
        rowmax(yc[0][q].y, yc[1][q].y, yc[2][q].y, b2, i2);
        float best = cb[q];
        int bi = ci[q];
        if (b1 > best) { best = b1; bi = 3 + i1; }
        if (b2 > best) { best = b2; bi = 6 + i2; }
        o[q] = f2bf(best);
        ai[q] = (uint8_t)bi;
        cb[q] = b2;   // this window's last row starts the next one
        ci[q] = i2;
      }
      const long long yo = (((long long)nu * OH + oh) * OW + owu) * C + c0;
      *(uint4*)(y + yo) = *(const uint4*)o;
      *(uint2*)(argmax + yo) = *(const uint2*)ai;
      if constexpr (PF) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          a[c] = na[c];
          b[c] = nb[c];
        }
      }
    }
  }
}

// The same walk with the channel halo taken from the neighbour lanes: a wave
// holds bpw = 64 / CV whole output-column units (its lanes the consecutive
// 8-channel chunks of one unit; the last 64 % CV lanes idle), so a pixel's
// channels c0 - 2, c0 - 1 are the lane below's mid.w and c0 + 8, c0 + 9 the
// lane above's mid.x: one 16-B load per pixel and two DPP moves instead of a
// 16-B and two 4-B loads (the walk is bound by its load stream, not by its
// log2 / exp2: profiles/r6/lrn_fwd_no_transcendentals_r6ff.txt).  Every lane
// runs R rows (the units of a wave may end their strips at different rows:
// rows past a unit's strip read clamped rows and store nothing), so every
// DPP move is wave-uniform.  Bit-identical to the walk.
__device__ __forceinline__ uint32_t dpp_from_below(uint32_t v) {  // lane - 1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf,
                                               true);
}
__device__ __forceinline__ uint32_t dpp_from_above(uint32_t v) {  // lane + 1
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf,
                                               true);
}

template <int half>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
void lrn_pool3s2_fwd_dpp_kernel(
    const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
    uint8_t* __restrict__ argmax, int N, int H, int W, int C, int OH, int OW,
    int R, int S, float alpha, float beta, float k, int bpw, int nunits,
    FastDiv fOW, FastDiv fS) {
  static_assert(half >= 1 && half <= 2, "dword halo");
  const int CV = C >> 3;
  const int lane = threadIdx.x & 63;
  const int lb = lane / CV, cvu = lane - lb * CV;
  const int c0 = cvu * 8;
  const bool has_lo = cvu > 0, has_hi = cvu < CV - 1;
  const uint32_t WC = (uint32_t)W * C, HWC = (uint32_t)H * WC;
  const uint32_t lastrow = (uint32_t)(H - 1) * WC;
  const int nwv = (nunits + bpw - 1) / bpw;
  const int wstride = (gridDim.x * blockDim.x) >> 6;
  // the loop bound is wave-uniform: every lane reaches every DPP move
  for (int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; wv < nwv;
       wv += wstride) {
    const int unit = wv * bpw + lb;
    const bool ok = lb < bpw && unit < nunits;
    uint32_t t2, owu, nu, su;
    fdivmod((uint32_t)(ok ? unit : 0), fOW, t2, owu);
    fdivmod(t2, fS, nu, su);
    const int w0 = (int)owu * 2;
    const int oh0 = (int)su * R, oh1 = min(OH, oh0 + R);
    const uint16_t* img = x + nu * HWC;
    const uint32_t col[3] = {(uint32_t)w0 * C, (uint32_t)(w0 + 1) * C,
                             (uint32_t)(w0 + 2) * C};
    auto ld = [&](uint32_t ro, int j) -> uint4 {
      return *(const uint4*)(img + ro + col[j] + c0);
    };
    auto halo = [&](const uint4& m) {
      LrnPx r;
      r.mid = m;
      const uint32_t lo = dpp_from_below(m.w), hi = dpp_from_above(m.x);
      r.lo = has_lo ? lo : 0u;
      r.hi = has_hi ? hi : 0u;
      return r;
    };
    auto rowmax = [&](float y0, float y1v, float y2v, float& b, int& bi) {
      b = y0;
      bi = 0;
      if (y1v > b) { b = y1v; bi = 1; }
      if (y2v > b) { b = y2v; bi = 2; }
    };
    float cb[8];
    int ci[8];
    {   // the strip's first window row
      const uint32_t ro = 2u * oh0 * WC;
      const LrnPx p0 = halo(ld(ro, 0)), p1 = halo(ld(ro, 1)),
                  p2 = halo(ld(ro, 2));
      f32x2v ya[8], yb[8];
      lrn_pair<half>(p0, p1, alpha, beta, k, ya);
      lrn_pair<half>(p2, p2, alpha, beta, k, yb);
#pragma unroll
      for (int q = 0; q < 8; ++q) rowmax(ya[q].x, ya[q].y, yb[q].x, cb[q], ci[q]);
    }
    uint4 a[3], b[3];
    auto load_rows = [&](int oh, uint4* ra, uint4* rb) {
      const uint32_t r1 = (uint32_t)(2 * oh + 1) * WC;
      const uint32_t hc1 = min(r1, lastrow), hc2 = min(r1 + WC, lastrow);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        ra[j] = ld(hc1, j);
        rb[j] = ld(hc2, j);
      }
    };
    load_rows(min(oh0, OH - 1), a, b);
    for (int r = 0; r < R; ++r) {
      const int oh = oh0 + r;
      uint4 na[3], nb[3];
      load_rows(min(oh + 1, OH - 1), na, nb);
      f32x2v yc[3][8];
#pragma unroll
      for (int c = 0; c < 3; ++c)
        lrn_pair<half>(halo(a[c]), halo(b[c]), alpha, beta, k, yc[c]);
      uint16_t o[8];
      uint8_t ai[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float b1, b2;
        int i1, i2;
        rowmax(yc[0][q].x, yc[1][q].x, yc[2][q].x, b1, i1);
        rowmax(yc[0][q].y, yc[1][q].y, yc[2][q].y, b2, i2);
        float best = cb[q];
        int bi = ci[q];
        if (b1 > best) { best = b1; bi = 3 + i1; }
        if (b2 > best) { best = b2; bi = 6 + i2; }
        o[q] = f2bf(best);
        ai[q] = (uint8_t)bi;
        cb[q] = b2;
        ci[q] = i2;
      }
      if (ok && oh < oh1) {
        const long long yo = (((long long)nu * OH + oh) * OW + owu) * C + c0;
        *(uint4*)(y + yo) = *(const uint4*)o;
        *(uint2*)(argmax + yo) = *(const uint2*)ai;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        a[c] = na[c];
        b[c] = nb[c];
      }
    }
  }
}

template <int half>
__global__ __launch_bounds__(256) void lrn_pool3s2_bwd_u8_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dp,
    const uint8_t* __restrict__ argmax, uint16_t* __restrict__ dx, int N,
    int H, int W, int C, int OH, int OW, float alpha, float beta, float k,
    const uint16_t* aux, int aux_act, FastDiv fCV, FastDiv fBW,
    FastDiv fBH) {
  // g[p][j]: pool gradient of block pixel p at channel c0 - 8 + j; only
  // j in [8 - half, 16 + half) is ever needed (the LRN window)
  constexpr int JLO = 8 - half, JHI = 16 + half;
  const int CV = C >> 3;
  const int BH = (H + 1) >> 1, BW = (W + 1) >> 1;
  const int total = N * BH * BW * CV;
  const bool aux_x = aux == x;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += gridDim.x * blockDim.x) {
    uint32_t blk, cvu, t, bwu, nu, bhu;
    fdivmod((uint32_t)e, fCV, blk, cvu);
    fdivmod(blk, fBW, t, bwu);
    fdivmod(t, fBH, nu, bhu);
    const int c0 = (int)cvu * 8;
    float g[4][24];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < 24; ++j) g[p][j] = 0.f;
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const int a = wi >> 1, b = wi & 1;
      const int oh = (int)bhu - 1 + a, ow = (int)bwu - 1 + b;
      if (oh < 0 || ow < 0 || oh >= OH || ow >= OW) continue;
      const long long yo = (((long long)nu * OH + oh) * OW + ow) * C;
#pragma unroll
      for (int part = 0; part < 3; ++part) {
        // channel chunk [c0 - 8 + 8 part, +8): skip chunks outside C and
        // those the LRN window never reaches
        if (8 * part + 8 <= JLO || 8 * part >= JHI) continue;
        const int cb = c0 - 8 + 8 * part;
        if (cb < 0 || cb >= C) continue;
        const uint4 gv = *(const uint4*)(dp + yo + cb);
        const uint2 av = *(const uint2*)(argmax + yo + cb);
        const uint16_t* gh = (const uint16_t*)&gv;
        const uint8_t* ah = (const uint8_t*)&av;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int r = 2 * (1 - a) + (p >> 1), c = 2 * (1 - b) + (p & 1);
          if (r > 2 || c > 2) continue;  // pixel outside this window
          const int kexp = r * 3 + c;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int j = 8 * part + q;
            if (j < JLO || j >= JHI) continue;
            g[p][j] += ah[q] == kexp ? bf2f(gh[q]) : 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int hp = (int)bhu * 2 + (p >> 1), wp = (int)bwu * 2 + (p & 1);
      if (hp >= H || wp >= W) continue;
      const long long po = (((long long)nu * H + hp) * W + wp) * C;
      float xv[24];
      loadx<half>(x + po, c0, C, xv);
      // t_j = g_j x_j s_j^(-beta-1) for j in [8 - half, 16 + half)
      float tj[24], sb[8];
#pragma unroll
      for (int j = JLO; j < JHI; ++j) {
        const float s = lrn_s(xv, j, half, alpha, k);
        const float e1 = ex2((-beta - 1.f) * __log2f(s));  // s^(-beta-1)
        tj[j] = g[p][j] * xv[j] * e1;
        if (j >= 8 && j < 16) sb[j - 8] = e1 * s;  // s^-beta
      }
      float av8[8];
      if (aux && !aux_x) load8(aux + po + c0, av8);
      uint16_t o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float acc = 0.f;
#pragma unroll
        for (int d = -half; d <= half; ++d) acc += tj[8 + q + d];
        float v = g[p][8 + q] * sb[q] - 2.f * alpha * beta * xv[8 + q] * acc;
        if (aux) v *= act_bwd(aux_x ? xv[8 + q] : av8[q], aux_act);
        o[q] = f2bf(v);
      }
      *(uint4*)(dx + po + c0) = *(const uint4*)o;
    }
  }
}

// The same backward with the LRN window halo shared across lanes.  Lanes of a
// wave hold consecutive 8-channel chunks of one 2 x 2 pixel block (64 / CV
// whole blocks per wave, the last 64 % CV lanes idle), so the channels a
// chunk's LRN window reaches beyond its own 8 - the squares x^2 for the
// window sums and the t_j = g_j x_j s_j^(-beta-1) terms of the gradient sum -
// are the neighbouring lanes' own values: one DPP wave shift each instead of
// loading, pooling-gradient-gathering and exponentiating 2 * half extra
// channels per pixel in every thread (the u8 kernel above does 12 channels'
// worth of transcendentals per 8 outputs at n = 5, this one 8).  AlexNet
// b512 on MI355X: conv1 0.337 -> 0.233 ms, conv2 0.215 -> 0.144 ms.  The
// same layout for the FORWARD kernel measured slower (conv1 0.194 ->
// 0.286 ms): its halo loads hit L1 and the DPP chains serialise 9 window
// pixels, so the forward keeps the per-thread halo.
__device__ __forceinline__ float lane_from_below(float v) {  // lane - 1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
      0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float lane_from_above(float v) {  // lane + 1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
      0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

// AM: the fused activation derivative, resolved at compile time (a runtime
// switch per pixel put a branch ladder between the four pixels of an
// iteration): 0 none, 1 strict ReLU of x itself (aux == x, the AlexNet
// conv -> LRN pair), 2 any (runtime aux / aux_act)
template <int half, bool PRE, int AM = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
void lrn_pool3s2_bwd_dpp_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dp,
    const uint8_t* __restrict__ argmax, uint16_t* __restrict__ dx, int N,
    int H, int W, int C, int OH, int OW, float alpha, float beta, float k,
    const uint16_t* aux, int aux_act, int bpw, int nblk, FastDiv fBW,
    FastDiv fBH) {
  const int CV = C >> 3;
  const int lane = threadIdx.x & 63;
  const int lb = lane / CV, cvu = lane - lb * CV;
  const int c0 = cvu * 8;
  const bool first = cvu == 0, last = cvu == CV - 1;
  const bool aux_x = aux == x;
  const int nwv = (nblk + bpw - 1) / bpw;
  const int wstride = (gridDim.x * blockDim.x) >> 6;
  // 32-bit element offsets (the host checks N H W C < 2^31): a handful of
  // multiplies per iteration instead of a 64-bit chain per load
  const uint32_t WC = (uint32_t)W * C, OWC = (uint32_t)OW * C;
  const uint32_t HWC = (uint32_t)H * WC, OHWC = (uint32_t)OH * OWC;
  // the loop bound is wave-uniform: every lane reaches every DPP
  for (int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; wv < nwv;
       wv += wstride) {
    const int blk = wv * bpw + lb;
    const bool ok = lb < bpw && blk < nblk;
    uint32_t t, bwu, nu, bhu;
    fdivmod((uint32_t)(ok ? blk : 0), fBW, t, bwu);
    fdivmod(t, fBH, nu, bhu);
    float g[4][8];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 8; ++q) g[p][q] = 0.f;
    // PRE: every load of the iteration (4 windows' gradient + argmax, 4
    // pixels of x) issued before any arithmetic, at clamped in-range
    // addresses - one memory round trip per iteration instead of one per
    // window and pixel
    uint4 gvv[4], xr[4];
    uint2 avv[4];
    // pixel p of the block: row 2 bh + (p >> 1), column 2 bw + (p & 1)
    // (clamped into the image; 2 bh < H always)
    const uint32_t xo = nu * HWC + c0;
    const uint32_t xrow[2] = {2 * bhu * WC, min(2 * bhu + 1, (uint32_t)H - 1) * WC};
    const uint32_t xcol[2] = {2 * bwu * (uint32_t)C,
                              min(2 * bwu + 1, (uint32_t)W - 1) * (uint32_t)C};
    if constexpr (PRE) {
      // windows (bh - 1 + a, bw - 1 + b), clamped
      const uint32_t yo0 = nu * OHWC + c0;
      const uint32_t yrow[2] = {(bhu > 0 ? bhu - 1 : 0) * OWC,
                                min(bhu, (uint32_t)OH - 1) * OWC};
      const uint32_t ycol[2] = {(bwu > 0 ? bwu - 1 : 0) * (uint32_t)C,
                                min(bwu, (uint32_t)OW - 1) * (uint32_t)C};
      const bool rok[2] = {bhu > 0, bhu < (uint32_t)OH};
      const bool cok[2] = {bwu > 0, bwu < (uint32_t)OW};
#pragma unroll
      for (int wi = 0; wi < 4; ++wi) {
        const int a = wi >> 1, b = wi & 1;
        const bool wv_ok = ok && rok[a] && cok[b];
        const uint32_t yo = yo0 + yrow[a] + ycol[b];
        gvv[wi] = *(const uint4*)(dp + yo);
        const uint2 av = *(const uint2*)(argmax + yo);
        // an absent window matches no pixel (index 0xff)
        avv[wi] = wv_ok ? av : make_uint2(0xffffffffu, 0xffffffffu);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
        xr[p] = *(const uint4*)(x + xo + xrow[p >> 1] + xcol[p & 1]);
    }
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const int a = wi >> 1, b = wi & 1;
      uint4 gv;
      uint2 av;
      if constexpr (PRE) {
        gv = gvv[wi];
        av = avv[wi];
      } else {
        const int oh = (int)bhu - 1 + a, ow = (int)bwu - 1 + b;
        if (!ok || oh < 0 || ow < 0 || oh >= OH || ow >= OW) continue;
        const long long yo = (((long long)nu * OH + oh) * OW + ow) * C + c0;
        gv = *(const uint4*)(dp + yo);
        av = *(const uint2*)(argmax + yo);
      }
      const uint16_t* gh = (const uint16_t*)&gv;
      // window indices as 32-bit byte extracts (a byte view of the uint2
      // compiled to 64-bit shifts and compares)
      uint32_t ai[8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        ai[q] = ((q < 4 ? av.x : av.y) >> (8 * (q & 3))) & 0xffu;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int r = 2 * (1 - a) + (p >> 1), c = 2 * (1 - b) + (p & 1);
        if (r > 2 || c > 2) continue;  // pixel outside this window
        const uint32_t kexp = r * 3 + c;
#pragma unroll
        for (int q = 0; q < 8; ++q) g[p][q] += ai[q] == kexp ? bf2f(gh[q]) : 0.f;
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int hp = (int)bhu * 2 + (p >> 1), wp = (int)bwu * 2 + (p & 1);
      const bool pv = ok && hp < H && wp < W;
      // (equal to the clamped offset whenever pv)
      const uint32_t po = xo + xrow[p >> 1] + xcol[p & 1];
      float xv[8];
      if constexpr (PRE) {
        // a pixel past the image edge (odd H / W) or of an absent block
        // reads a clamped in-range pixel: its values reach no valid lane (the
        // DPP halo stops at block edges, no window selects it) and it is not
        // stored
        const uint16_t* h8 = (const uint16_t*)&xr[p];
#pragma unroll
        for (int q = 0; q < 8; ++q) xv[q] = bf2f(h8[q]);
      } else if (pv) {
        load8(x + po, xv);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) xv[q] = 0.f;
      }
      // The kernel is VALU-bound (~87 % of SIMD cycles at AlexNet conv1
      // b1024): the per-channel products run on channel pairs (f32x2_t ->
      // v_pk_mul_f32 / v_pk_fma_f32, two lanes' worth per instruction) and
      // the (2 half + 1)-term window sums slide (w_{q+1} = w_q + e_{q+2h+1}
      // - e_q: 2 ops per output instead of 2 half)
      f32x2_t X2[4], G2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        X2[i] = f32x2_t{xv[2 * i], xv[2 * i + 1]};
        G2[i] = f32x2_t{g[p][2 * i], g[p][2 * i + 1]};
      }
      if constexpr (AM == 1) {
        // x is the ReLU output (>= 0): dx = 0 where x = 0 is g = 0 there
        // (that channel's t_j = g x s^(-beta-1) is 0 anyway) - one clamped
        // product per channel pair, min(max(x 2^126, 0), 1) = [x > 0] for
        // every normal x, instead of a compare and a select per channel
        // (the compiler splits a clamped vector product into two scalar
        // v_max clamps; the packed product's clamp bit does it in one)
        const f32x2_t BIG = {0x1p126f, 0x1p126f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x2_t m;
          asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(m) : "v"(X2[i]), "v"(BIG));
          G2[i] = G2[i] * m;
        }
      }
      // squares of channels c0 - half .. c0 + 8 + half
      float e[8 + 2 * half];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2_t sq2 = X2[i] * X2[i];
        e[half + 2 * i] = sq2.x;
        e[half + 2 * i + 1] = sq2.y;
      }
#pragma unroll
      for (int d = 0; d < half; ++d) {
        const float lo = lane_from_below(e[8 + d]);   // its channel 8-half+d
        const float hi = lane_from_above(e[half + d]);  // its channel d
        e[d] = first ? 0.f : lo;
        e[8 + half + d] = last ? 0.f : hi;
      }
      float w[8];
      w[0] = e[0];
#pragma unroll
      for (int d = 1; d <= 2 * half; ++d) w[0] += e[d];
#pragma unroll
      for (int q = 1; q < 8; ++q) w[q] = (w[q - 1] + e[q + 2 * half]) - e[q - 1];
      // Scaled by c = 2 alpha beta (> 0: the host routes alpha beta = 0 to
      // the per-thread kernel): S = s / c, E = c s^(-beta-1) (the log2 c
      // terms fold into one fma), so E S = s^-beta, T = c t_j and
      // dx = g s^-beta - x sum(T) - no separate product by -2 alpha beta
      const float cs = 2.f * alpha * beta;
      const f32x2_t K2 = {k / cs, k / cs}, A2 = {0.5f / beta, 0.5f / beta};
      const f32x2_t NB1 = {-beta - 1.f, -beta - 1.f};
      const float lc = -beta * __log2f(cs);
      const f32x2_t LC2 = {lc, lc};
      f32x2_t SB2[4], T2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2_t S2 = K2 + A2 * f32x2_t{w[2 * i], w[2 * i + 1]};
        const f32x2_t L2 = f32x2_t{__log2f(S2.x), __log2f(S2.y)} * NB1 + LC2;
        const f32x2_t E2 = {ex2(L2.x), ex2(L2.y)};  // c s^(-beta-1)
        SB2[i] = E2 * S2;                               // s^-beta
        T2[i] = G2[i] * X2[i] * E2;                     // c t_j
      }
      float tj[8 + 2 * half];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        tj[half + 2 * i] = T2[i].x;
        tj[half + 2 * i + 1] = T2[i].y;
      }
#pragma unroll
      for (int d = 0; d < half; ++d) {
        const float lo = lane_from_below(tj[8 + d]);
        const float hi = lane_from_above(tj[half + d]);
        tj[d] = first ? 0.f : lo;
        tj[8 + half + d] = last ? 0.f : hi;
      }
      float acc[8];
      acc[0] = tj[0];
#pragma unroll
      for (int d = 1; d <= 2 * half; ++d) acc[0] += tj[d];
#pragma unroll
      for (int q = 1; q < 8; ++q)
        acc[q] = (acc[q - 1] + tj[q + 2 * half]) - tj[q - 1];
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2_t V2 =
            G2[i] * SB2[i] - X2[i] * f32x2_t{acc[2 * i], acc[2 * i + 1]};
        v[2 * i] = V2.x;
        v[2 * i + 1] = V2.y;
      }
      if constexpr (AM == 2) {
        if (aux && pv) {
          float av8[8];
          if (aux_x) {
#pragma unroll
            for (int q = 0; q < 8; ++q) av8[q] = xv[q];
          } else {
            load8(aux + po, av8);
          }
          act_bwd_mul8(v, av8, aux_act);
        }
      }
      if (pv) *(uint4*)(dx + po) = pack_bf16x8(v);
    }
  }
}
}  // namespace

// Stochastic pooling (Znicz stochastic_pooling / stochastic_abs_pooling):
// each window element is drawn with probability w_i / sum(w), w = max(x, 0)
// (|x| for abs), uniform over the window when sum(w) = 0; the uniform of
// output element o is hash(o, seed) >> 8 / 2^24 (counter-based, the seed read
// from device memory so a captured step draws fresh samples every replay).
// Testing: the probability-weighted average, argmax = the most probable.
// One thread per output element (channels fastest: coalesced).
__device__ __forceinline__ uint32_t sp_hash(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__global__ void stochastic_pool_kernel(const uint16_t* __restrict__ x,
                                       uint16_t* __restrict__ y,
                                       int* __restrict__ argmax, int N, int H,
                                       int W, int C, int OH, int OW, int ky,
                                       int kx, int sy, int sx, int use_abs,
                                       int train, const uint32_t* seed_dev,
                                       FastDiv fC, FastDiv fOW, FastDiv fOH) {
  const uint32_t seed = __builtin_amdgcn_readfirstlane(seed_dev[0]);
  const long long total = (long long)N * OH * OW * C;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       o < total; o += (long long)gridDim.x * blockDim.x) {
    uint32_t pix, c, t, ow, n, oh;
    fdivmod((uint32_t)o, fC, pix, c);
    fdivmod(pix, fOW, t, ow);
    fdivmod(t, fOH, n, oh);
    const int h0 = (int)oh * sy, w0 = (int)ow * sx;
    const int h1 = min(h0 + ky, H), w1 = min(w0 + kx, W);
    const long long img = (long long)n * H * W * C + c;
    float tot = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        const float v = bf2f(x[img + ((long long)h * W + w) * C]);
        tot += use_abs ? fabsf(v) : fmaxf(v, 0.f);
      }
    const int cnt = (h1 - h0) * (w1 - w0);
    const float inv = tot > 0.f ? 1.f / tot : 0.f;
    const float uni = 1.f / (float)cnt;
    const float u =
        (float)(sp_hash((uint32_t)o, seed) >> 8) * (1.f / 16777216.f);
    float cum = 0.f, out = 0.f, best = -1.f;
    long long pick = -1;
    bool taken = false;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) {
        const long long off = img + ((long long)h * W + w) * C;
        const float v = bf2f(x[off]);
        const float pr = tot > 0.f ? (use_abs ? fabsf(v) : fmaxf(v, 0.f)) * inv
                                   : uni;
        if (train) {
          cum += pr;
          if (!taken && cum >= u) { taken = true; pick = off; out = v; }
          if (!taken) { pick = off; out = v; }  // rounding: the last one
        } else {
          out += pr * v;
          if (pr > best) { best = pr; pick = off; }
        }
      }
    y[o] = f2bf(out);
    argmax[o] = (int)pick;
  }
}

HVK_API int hvk_stochastic_pool(const void* x, void* y, int* argmax, int N,
                                int H, int W, int C, int OH, int OW, int ky,
                                int kx, int sy, int sx, int use_abs, int train,
                                const void* seed_dev, hipStream_t s) {
  const long long total = (long long)N * OH * OW * C;
  if ((long long)N * H * W * C >= (1ll << 31) || !seed_dev) return -1;
  hipLaunchKernelGGL(stochastic_pool_kernel, dim3(grid_for(total)), dim3(256),
                     0, s, (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W,
                     C, OH, OW, ky, kx, sy, sx, use_abs, train,
                     (const uint32_t*)seed_dev, make_fastdiv(C),
                     make_fastdiv(OW), make_fastdiv(OH));
  return (int)launch_status(s);
}

// 2 x 2 / stride-2 pooling without argmax (pool2_fwd_kernel): C % 8 == 0,
// even H and W, 16-B aligned tensors; mode 0 max, 1 avg, 2 maxabs.
// q8 / q8_st / q8_shard / q8_fmax / q8_fmt / hist (q8 may be null): the
// fused fp8 copy of the result for the next fp8 layer (fp8_common.h Q8)
HVK_API int hvk_pool2_fwd_q8(const void* x, void* y, int N, int H, int W,
                             int C, int mode, void* q8, const float* q8_st,
                             float* q8_shard, float q8_fmax, int q8_fmt,
                             int hist, hipStream_t s) {
  if (C % 8 || (H & 1) || (W & 1) || ((uintptr_t)x & 15) ||
      ((uintptr_t)y & 15) || ((uintptr_t)q8 & 7) ||
      (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const Q8 q{(uint8_t*)q8, q8_st, q8_shard, q8_fmax, q8_fmt, hist};
  const long long total = (long long)N * (H / 2) * (W / 2) * (C / 8);
  auto k = mode == POOL_AVG ? pool2_fwd_kernel<POOL_AVG>
           : mode == POOL_MAXABS ? pool2_fwd_kernel<POOL_MAXABS>
                                 : pool2_fwd_kernel<POOL_MAX>;
  hipLaunchKernelGGL(k, dim3(grid_for(total)), dim3(256), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, N, H, W, C,
                     make_fastdiv(C / 8), make_fastdiv(W / 2),
                     make_fastdiv(H / 2), q);
  return (int)launch_status(s);
}

HVK_API int hvk_pool2_fwd(const void* x, void* y, int N, int H, int W, int C,
                          int mode, hipStream_t s) {
  return hvk_pool2_fwd_q8(x, y, N, H, W, C, mode, nullptr, nullptr, nullptr,
                          1.f, 0, 0, s);
}

// dx of a 2 x 2 / stride-2 pooling, the choice recomputed from x (the
// forward input); aux multiplies by act_bwd(aux) (aux may be x itself)
HVK_API int hvk_pool2_bwd_q8(const void* x, const void* dy, void* dx, int N,
                             int H, int W, int C, int mode, const void* aux,
                             int aux_act, void* q8, const float* q8_st,
                             float* q8_shard, float q8_fmax, int q8_fmt,
                             int hist, hipStream_t s) {
  if (C % 8 || (H & 1) || (W & 1) || ((uintptr_t)x & 15) ||
      ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15) || ((uintptr_t)aux & 15) ||
      ((uintptr_t)q8 & 7) || (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const Q8 q{(uint8_t*)q8, q8_st, q8_shard, q8_fmax, q8_fmt, hist};
  const long long total = (long long)N * (H / 2) * (W / 2) * (C / 8);
  auto k = mode == POOL_AVG ? pool2_bwd_kernel<POOL_AVG>
           : mode == POOL_MAXABS ? pool2_bwd_kernel<POOL_MAXABS>
                                 : pool2_bwd_kernel<POOL_MAX>;
  hipLaunchKernelGGL(k, dim3(grid_for(total)), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)dy, (uint16_t*)dx,
                     N, H, W, C, (const uint16_t*)aux, aux_act,
                     make_fastdiv(C / 8), make_fastdiv(W / 2),
                     make_fastdiv(H / 2), q);
  return (int)launch_status(s);
}

HVK_API int hvk_pool2_bwd(const void* x, const void* dy, void* dx, int N,
                          int H, int W, int C, int mode, const void* aux,
                          int aux_act, hipStream_t s) {
  return hvk_pool2_bwd_q8(x, dy, dx, N, H, W, C, mode, aux, aux_act, nullptr,
                          nullptr, nullptr, 1.f, 0, 0, s);
}

// forward kernel selector for A/B runs (hvk_set_lrn_fwd_variant): 0 the
// vertical walk with the next row prefetched and DPP channel halos (round
// 6), 5 the same walk loading its halos, 1 the per-output preloading
// kernel, 2 the walk without the prefetch, 3 / 4 the walk with the prefetch
// over strips of about 5 / 9 output rows (0 / 5: about 14; AlexNet b2048,
// tools/bench_lrn.py: conv2 273 -> 256 us from 9 to 14, conv1 419 / 423,
// 5 rows 469 / 287: profiles/r4/lrn_fwd_strips_b2048.json)
static int g_lrn_fwd_variant = 0;
HVK_API void hvk_set_lrn_fwd_variant(int v) { g_lrn_fwd_variant = v; }
// backward selector (hvk_set_lrn_bwd_variant): 0 every load of an
// iteration issued first, 1 loads next to their use
static int g_lrn_bwd_variant = 0;
HVK_API void hvk_set_lrn_bwd_variant(int v) { g_lrn_bwd_variant = v; }

// Fused LRN -> 3x3 stride-2 max pooling with a uint8 window-index argmax
// (see lrn_pool3s2_fwd_u8_kernel).  C % 8 == 0, n / 2 <= 4.
HVK_API int hvk_lrn_pool_fwd_u8(const void* x, void* y, void* argmax, int N,
                                int H, int W, int C, int OH, int OW, int n,
                                float alpha, float beta, float k,
                                hipStream_t s) {
  if (C % 8 || n / 2 > 4 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15) ||
      ((uintptr_t)argmax & 7) || (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const int h = n / 2;
  const long long total = (long long)N * OH * OW * (C / 8);
  if (h >= 1 && h <= 2 && g_lrn_fwd_variant == 0 && C / 8 <= 64 &&
      OH == (H - 3) / 2 + 1 && OW == (W - 3) / 2 + 1) {
    // the walk with DPP channel halos (whole output-column units per wave):
    // AlexNet b3072 conv1 611 -> 581 us, conv2 362 -> 337 us, bit-identical
    // (tools/bench_lrn.py, profiles/r6/bench_lrn_dpp_halo_r6gg.log)
    const int t = 14;
    const int S = (OH + t - 1) / t, R = (OH + S - 1) / S;
    const int CV = C / 8, bpw = 64 / CV;
    const long long nunits = (long long)N * S * OW;
    const long long waves = (nunits + bpw - 1) / bpw;
    auto kd = h == 1 ? lrn_pool3s2_fwd_dpp_kernel<1>
                     : lrn_pool3s2_fwd_dpp_kernel<2>;
    hipLaunchKernelGGL(kd, dim3(grid_for(waves * 64)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, (uint8_t*)argmax, N,
                       H, W, C, OH, OW, R, S, alpha, beta, k, bpw,
                       (int)nunits, make_fastdiv(OW), make_fastdiv(S));
    return (int)launch_status(s);
  }
  if (h >= 1 && h <= 2 && g_lrn_fwd_variant != 1 && OH == (H - 3) / 2 + 1 &&
      OW == (W - 3) / 2 + 1) {
    // vertical walk over strips of about 14 output rows (AlexNet: one strip
    // for conv2's 13 rows, two for conv1's 27)
    const int t = g_lrn_fwd_variant == 3 ? 5 : g_lrn_fwd_variant == 4 ? 9 : 14;
    const int S = (OH + t - 1) / t, R = (OH + S - 1) / S;
    const long long tw = (long long)N * S * OW * (C / 8);
    const bool pf = g_lrn_fwd_variant != 2;   // (5: this walk, prefetched)
    auto kw = h == 1 ? (pf ? lrn_pool3s2_fwd_walk_kernel<1, true>
                           : lrn_pool3s2_fwd_walk_kernel<1, false>)
                     : (pf ? lrn_pool3s2_fwd_walk_kernel<2, true>
                           : lrn_pool3s2_fwd_walk_kernel<2, false>);
    hipLaunchKernelGGL(kw, dim3(grid_for(tw)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, (uint8_t*)argmax, N,
                       H, W, C, OH, OW, R, S, alpha, beta, k,
                       make_fastdiv(C / 8), make_fastdiv(OW), make_fastdiv(S));
    return (int)launch_status(s);
  }
  if (h >= 1 && h <= 2) {
    auto kp = h == 1 ? lrn_pool3s2_fwd_u8p_kernel<1>
                     : lrn_pool3s2_fwd_u8p_kernel<2>;
    hipLaunchKernelGGL(kp, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, (uint8_t*)argmax, N,
                       H, W, C, OH, OW, alpha, beta, k, make_fastdiv(C / 8),
                       make_fastdiv(OW), make_fastdiv(OH));
    return (int)launch_status(s);
  }
  auto kf = h == 0 ? lrn_pool3s2_fwd_u8_kernel<0>
          : h == 1 ? lrn_pool3s2_fwd_u8_kernel<1>
          : h == 2 ? lrn_pool3s2_fwd_u8_kernel<2>
          : h == 3 ? lrn_pool3s2_fwd_u8_kernel<3>
                   : lrn_pool3s2_fwd_u8_kernel<4>;
  hipLaunchKernelGGL(kf, dim3(grid_for(total)), dim3(256), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, (uint8_t*)argmax, N, H,
                     W, C, OH, OW, alpha, beta, k, make_fastdiv(C / 8),
                     make_fastdiv(OW), make_fastdiv(OH));
  return (int)launch_status(s);
}

HVK_API int hvk_lrn_pool_bwd_u8(const void* x, const void* dp,
                                const void* argmax, void* dx, int N, int H,
                                int W, int C, int OH, int OW, int n,
                                float alpha, float beta, float k,
                                const void* aux, int aux_act, hipStream_t s) {
  if (C % 8 || n / 2 > 4 || ((uintptr_t)x & 15) || ((uintptr_t)dp & 15) ||
      ((uintptr_t)dx & 15) || ((uintptr_t)argmax & 7) ||
      ((uintptr_t)aux & 15) || (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const int h = n / 2;
  const int BH = (H + 1) / 2, BW = (W + 1) / 2;
  const long long tb = (long long)N * BH * BW * (C / 8);
  if (C / 8 <= 64 && h >= 1 && h <= 4 && alpha * beta > 0.f && k > 0.f) {
    // whole 2 x 2 blocks per wave, their chunks on consecutive lanes
    const int CV = C / 8, bpw = 64 / CV;
    const long long nblk = (long long)N * BH * BW;
    const long long waves = (nblk + bpw - 1) / bpw;
    const long long blocks = std::min<long long>((waves + 3) / 4, 1 << 16);
    const bool pre = g_lrn_bwd_variant == 0;
    // the activation derivative as a template: none, ReLU of x, any
    const int am = !aux ? 0 : (aux == x && aux_act == ACT_STRICT_RELU) ? 1 : 2;
#define LRN_BWD_K(H)                                                      \
    (!pre      ? lrn_pool3s2_bwd_dpp_kernel<H, false>                     \
     : am == 0 ? lrn_pool3s2_bwd_dpp_kernel<H, true, 0>                   \
     : am == 1 ? lrn_pool3s2_bwd_dpp_kernel<H, true, 1>                   \
               : lrn_pool3s2_bwd_dpp_kernel<H, true, 2>)
    auto kd = h == 1 ? LRN_BWD_K(1) : h == 2 ? LRN_BWD_K(2)
            : h == 3 ? LRN_BWD_K(3) : LRN_BWD_K(4);
#undef LRN_BWD_K
    hipLaunchKernelGGL(kd, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const uint16_t*)x, (const uint16_t*)dp,
                       (const uint8_t*)argmax, (uint16_t*)dx, N, H, W, C, OH,
                       OW, alpha, beta, k, (const uint16_t*)aux, aux_act, bpw,
                       (int)nblk, make_fastdiv(BW), make_fastdiv(BH));
    return (int)launch_status(s);
  }
  auto k2 = h == 0 ? lrn_pool3s2_bwd_u8_kernel<0>
          : h == 1 ? lrn_pool3s2_bwd_u8_kernel<1>
          : h == 2 ? lrn_pool3s2_bwd_u8_kernel<2>
          : h == 3 ? lrn_pool3s2_bwd_u8_kernel<3>
                   : lrn_pool3s2_bwd_u8_kernel<4>;
  hipLaunchKernelGGL(k2, dim3(grid_for(tb)), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)dp,
                     (const uint8_t*)argmax, (uint16_t*)dx, N, H, W, C, OH, OW,
                     alpha, beta, k, (const uint16_t*)aux, aux_act,
                     make_fastdiv(C / 8), make_fastdiv(BW), make_fastdiv(BH));
  return (int)launch_status(s);
}

HVK_API int hvk_pool_fwd(const void* x, void* y, int* argmax, int N, int H,
                         int W, int C, int OH, int OW, int ky, int kx, int sy,
                         int sx, int pt, int pl, int mode, hipStream_t s) {
  if (C % 8 == 0 && ky == 3 && kx == 3 && ((uintptr_t)x & 15) == 0 &&
      ((uintptr_t)y & 15) == 0 && ((uintptr_t)argmax & 15) == 0 &&
      (long long)N * H * W * C < (1ll << 31)) {
    long long total = (long long)N * OH * OW * (C / 8);
    auto k = mode == POOL_AVG ? pool_fwd3_kernel<POOL_AVG>
             : mode == POOL_MAXABS ? pool_fwd3_kernel<POOL_MAXABS>
                                   : pool_fwd3_kernel<POOL_MAX>;
    hipLaunchKernelGGL(k, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C,
                       OH, OW, sy, sx, pt, pl, make_fastdiv(C / 8),
                       make_fastdiv(OW), make_fastdiv(OH));
  } else if (C % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    long long total = (long long)N * OH * OW * (C / 8);
    hipLaunchKernelGGL(pool_fwd_kernel<8>, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, make_fastdiv(C / 8),
                       make_fastdiv(OW), make_fastdiv(OH));
  } else {
    // C off the 8-grid (LeNet's 20 / 50): 4- or 2-channel lanes
    const int v = (C % 4 == 0 && ((uintptr_t)x & 7) == 0 &&
                   ((uintptr_t)y & 7) == 0) ? 4
                  : (C % 2 == 0 && ((uintptr_t)x & 3) == 0 &&
                     ((uintptr_t)y & 3) == 0) ? 2 : 1;
    long long total = (long long)N * OH * OW * (C / v);
    auto k = v == 4 ? pool_fwd_kernel<4> : v == 2 ? pool_fwd_kernel<2>
                                                  : pool_fwd_kernel<1>;
    hipLaunchKernelGGL(k, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, make_fastdiv(C / v),
                       make_fastdiv(OW), make_fastdiv(OH));
  }
  return (int)launch_status(s);
}

HVK_API int hvk_pool_bwd(const void* dy, const int* argmax, void* dx, int N,
                         int H, int W, int C, int OH, int OW, int ky, int kx,
                         int sy, int sx, int pt, int pl, int mode,
                         const void* aux, int aux_act, hipStream_t s) {
  if (C % 8 == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0 &&
      ((uintptr_t)aux & 15) == 0) {
    long long total = (long long)N * H * W * (C / 8);
    if (ky == 3 && kx == 3 && sy == 2 && sx == 2 && pt == 0 && pl == 0 &&
        mode != POOL_AVG && g_pool_bwd_variant == 0 &&
        ((uintptr_t)argmax & 15) == 0 &&
        (long long)N * H * W * C < (1ll << 31)) {
      const long long tb = (long long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
      auto kb = mode == POOL_MAXABS ? pool_bwd3s2_blk_kernel<POOL_MAXABS>
                                    : pool_bwd3s2_blk_kernel<POOL_MAX>;
      hipLaunchKernelGGL(kb, dim3(grid_for(tb)), dim3(256), 0, s,
                         (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W,
                         C, OH, OW, (const uint16_t*)aux, aux_act,
                         make_fastdiv(C / 8), make_fastdiv((W + 1) / 2),
                         make_fastdiv((H + 1) / 2));
      return (int)launch_status(s);
    }
    if (ky == 3 && kx == 3 && sy >= 2 && sx >= 2 &&
        ((uintptr_t)argmax & 15) == 0 &&
        (long long)N * H * W * C < (1ll << 31)) {
      auto k3 = mode == POOL_AVG ? pool_bwd3_kernel<POOL_AVG>
                                 : pool_bwd3_kernel<POOL_MAX>;
      hipLaunchKernelGGL(k3, dim3(grid_for(total)), dim3(256), 0, s,
                         (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W,
                         C, OH, OW, sy, sx, pt, pl, (const uint16_t*)aux,
                         aux_act, make_fastdiv(C / 8), make_fastdiv(W),
                         make_fastdiv(H), make_fastdiv(sy), make_fastdiv(sx));
      return (int)launch_status(s);
    }
    auto k8 = mode == POOL_AVG ? pool_bwd_kernel<8, POOL_AVG>
                               : pool_bwd_kernel<8, POOL_MAX>;
    hipLaunchKernelGGL(k8, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, (const uint16_t*)aux,
                       aux_act, make_fastdiv(C / 8), make_fastdiv(W),
                       make_fastdiv(H), make_fastdiv(sy), make_fastdiv(sx));
  } else {
    const uintptr_t al = (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)aux;
    const int v = (C % 4 == 0 && (al & 7) == 0) ? 4
                  : (C % 2 == 0 && (al & 3) == 0) ? 2 : 1;
    long long total = (long long)N * H * W * (C / v);
    auto k1 = v == 4 ? (mode == POOL_AVG ? pool_bwd_kernel<4, POOL_AVG>
                                         : pool_bwd_kernel<4, POOL_MAX>)
            : v == 2 ? (mode == POOL_AVG ? pool_bwd_kernel<2, POOL_AVG>
                                         : pool_bwd_kernel<2, POOL_MAX>)
                     : (mode == POOL_AVG ? pool_bwd_kernel<1, POOL_AVG>
                                         : pool_bwd_kernel<1, POOL_MAX>);
    hipLaunchKernelGGL(k1, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, (const uint16_t*)aux,
                       aux_act, make_fastdiv(C / v), make_fastdiv(W),
                       make_fastdiv(H), make_fastdiv(sy), make_fastdiv(sx));
  }
  return (int)launch_status(s);
}

HVK_API int hvk_lrn_fwd(const void* x, void* y, long long P, int C, int n,
                        float alpha, float beta, float k, hipStream_t s) {
  if (C % 8 == 0 && n / 2 <= 4 && P * C < (1ll << 31) &&
      ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    long long total = P * (C / 8);
    const int h = n / 2;
    auto kf = h == 0 ? lrn_fwd_vec_kernel<0> : h == 1 ? lrn_fwd_vec_kernel<1> : h == 2 ? lrn_fwd_vec_kernel<2>
            : h == 3 ? lrn_fwd_vec_kernel<3> : lrn_fwd_vec_kernel<4>;
    hipLaunchKernelGGL(kf, dim3(grid_for(total)), dim3(256), 0,
                       s, (const uint16_t*)x, (uint16_t*)y, (int)P, C,
                       alpha, beta, k, make_fastdiv(C / 8));
    return (int)launch_status(s);
  }
  if (C > 1024) return -1;
  hipLaunchKernelGGL(lrn_fwd_kernel, dim3(grid_for(P, 4)), dim3(256), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, P, C, n, alpha, beta, k);
  return (int)launch_status(s);
}

HVK_API int hvk_lrn_bwd(const void* x, const void* dy, void* dx, long long P,
                        int C, int n, float alpha, float beta, float k,
                        const void* aux, int aux_act, hipStream_t s) {
  if (C % 8 == 0 && n / 2 <= 4 && P * C < (1ll << 31) &&
      ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 &&
      ((uintptr_t)dx & 15) == 0 && ((uintptr_t)aux & 15) == 0) {
    long long total = P * (C / 8);
    const int h = n / 2;
    auto kb = h == 0 ? lrn_bwd_vec_kernel<0> : h == 1 ? lrn_bwd_vec_kernel<1> : h == 2 ? lrn_bwd_vec_kernel<2>
            : h == 3 ? lrn_bwd_vec_kernel<3> : lrn_bwd_vec_kernel<4>;
    hipLaunchKernelGGL(kb, dim3(grid_for(total)), dim3(256), 0,
                       s, (const uint16_t*)x, (const uint16_t*)dy,
                       (uint16_t*)dx, (int)P, C, alpha, beta, k,
                       (const uint16_t*)aux, aux_act, make_fastdiv(C / 8));
    return (int)launch_status(s);
  }
  if (C > 1024) return -1;
  hipLaunchKernelGGL(lrn_bwd_kernel, dim3(grid_for(P, 4)), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)dy, (uint16_t*)dx, P,
                     C, n, alpha, beta, k, (const uint16_t*)aux, aux_act);
  return (int)launch_status(s);
}

// Fused LRN (across channels) -> 3x3 max pooling (no padding, stride >= 2),
// C % 8 == 0, n / 2 <= 4.  y / argmax as hvk_pool_fwd applied to lrn(x).
HVK_API int hvk_lrn_pool_fwd(const void* x, void* y, int* argmax, int N,
                             int H, int W, int C, int OH, int OW, int sy,
                             int sx, int n, float alpha, float beta, float k,
                             hipStream_t s) {
  if (C % 8 || n / 2 > 4 || sy < 2 || sx < 2 || ((uintptr_t)x & 15) ||
      ((uintptr_t)y & 15) || ((uintptr_t)argmax & 15) ||
      (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const long long total = (long long)N * OH * OW * (C / 8);
  const int h = n / 2;
  auto kf = h == 0 ? lrn_pool3_fwd_kernel<0> : h == 1 ? lrn_pool3_fwd_kernel<1>
          : h == 2 ? lrn_pool3_fwd_kernel<2> : h == 3 ? lrn_pool3_fwd_kernel<3>
                   : lrn_pool3_fwd_kernel<4>;
  hipLaunchKernelGGL(kf, dim3(grid_for(total)), dim3(256), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C, OH,
                     OW, sy, sx, alpha, beta, k, make_fastdiv(C / 8),
                     make_fastdiv(OW), make_fastdiv(OH));
  return (int)launch_status(s);
}

// dx = lrn_bwd(x, pool_bwd(dp, argmax)) [* f'(aux)] in one pass
HVK_API int hvk_lrn_pool_bwd(const void* x, const void* dp, const int* argmax,
                             void* dx, int N, int H, int W, int C, int OH,
                             int OW, int sy, int sx, int n, float alpha,
                             float beta, float k, const void* aux,
                             int aux_act, hipStream_t s) {
  if (C % 8 || n / 2 > 4 || sy < 2 || sx < 2 || ((uintptr_t)x & 15) ||
      ((uintptr_t)dp & 15) || ((uintptr_t)dx & 15) ||
      ((uintptr_t)argmax & 15) || ((uintptr_t)aux & 15) ||
      (long long)N * H * W * C >= (1ll << 31))
    return -1;
  const int h = n / 2;
  if (sy == 2 && sx == 2) {
    const int BH = (H + 1) / 2, BW = (W + 1) / 2;
    const long long tb = (long long)N * BH * BW * (C / 8);
    auto k2 = h == 0 ? lrn_pool3s2_bwd_kernel<0>
            : h == 1 ? lrn_pool3s2_bwd_kernel<1>
            : h == 2 ? lrn_pool3s2_bwd_kernel<2>
            : h == 3 ? lrn_pool3s2_bwd_kernel<3> : lrn_pool3s2_bwd_kernel<4>;
    hipLaunchKernelGGL(k2, dim3(grid_for(tb)), dim3(256), 0, s,
                       (const uint16_t*)x, (const uint16_t*)dp, argmax,
                       (uint16_t*)dx, N, H, W, C, OH, OW, alpha, beta, k,
                       (const uint16_t*)aux, aux_act, make_fastdiv(C / 8),
                       make_fastdiv(BW), make_fastdiv(BH));
    return (int)launch_status(s);
  }
  const long long total = (long long)N * H * W * (C / 8);
  auto kb = h == 0 ? lrn_pool3_bwd_kernel<0> : h == 1 ? lrn_pool3_bwd_kernel<1>
          : h == 2 ? lrn_pool3_bwd_kernel<2> : h == 3 ? lrn_pool3_bwd_kernel<3>
                   : lrn_pool3_bwd_kernel<4>;
  hipLaunchKernelGGL(kb, dim3(grid_for(total)), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)dp, argmax,
                     (uint16_t*)dx, N, H, W, C, OH, OW, sy, sx, alpha, beta, k,
                     (const uint16_t*)aux, aux_act, make_fastdiv(C / 8),
                     make_fastdiv(W), make_fastdiv(H), make_fastdiv(sy),
                     make_fastdiv(sx));
  return (int)launch_status(s);
}
