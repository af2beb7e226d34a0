// pool_lrn.hip - NHWC pooling (max / avg / maxabs) and local response
// normalisation across channels, forward and backward, for gfx950.
//
// Replaces the (absent) Znicz pooling / gd_pooling / normalization kernels
// (docs/OPS.md).  Layout is NHWC so the channel vector of a
// pixel is contiguous: pooling threads own 8 channels (one 16-B bf16 load),
// LRN waves own one pixel and stage its channels in LDS.  Pooling backward is
// a deterministic GATHER (each input element sums the windows that chose it)
// instead of atomics.
#include "hvk_common.h"

using namespace hvk;

namespace {
inline int grid_for(long long n, int per_block = 256) {
  long long g = (n + per_block - 1) / per_block;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : (int)g;
}

enum PoolMode { POOL_MAX = 0, POOL_AVG = 1, POOL_MAXABS = 2 };

// one thread = one output pixel x 8 channels (C % 8 == 0) or x 1 channel
template <int VEC>
__global__ void pool_fwd_kernel(const uint16_t* x, uint16_t* y, int* argmax,
                                int N, int H, int W, int C, int OH, int OW,
                                int ky, int kx, int sy, int sx, int pt, int pl,
                                int mode) {
  const int CV = C / VEC;
  long long total = (long long)N * OH * OW * CV;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int cv = (int)(e % CV);
    long long pix = e / CV;
    int ow = (int)(pix % OW);
    long long t = pix / OW;
    int oh = (int)(t % OH);
    int n = (int)(t / OH);
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
        long long off = (((long long)n * H + h) * W + w) * C + cv * VEC;
        uint16_t v[VEC];
        if (VEC == 8) *(uint4*)v = *(const uint4*)(x + off);
        else v[0] = x[off];
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          float f = bf2f(v[q]);
          if (mode == POOL_AVG) {
            sum[q] += f;
          } else {
            float key = mode == POOL_MAXABS ? fabsf(f) : f;
            float bk = mode == POOL_MAXABS ? fabsf(best[q]) : best[q];
            if (bidx[q] < 0 || key > bk) { best[q] = f; bidx[q] = (int)(off + q); }
          }
        }
      }
    int cnt = (h1 - h0) * (w1 - w0);
    uint16_t o[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      o[q] = f2bf(mode == POOL_AVG ? sum[q] / (float)max(cnt, 1) : best[q]);
    long long yo = pix * C + cv * VEC;
    if (VEC == 8) *(uint4*)(y + yo) = *(uint4*)o;
    else y[yo] = o[0];
    if (argmax && mode != POOL_AVG) {
#pragma unroll
      for (int q = 0; q < VEC; ++q) argmax[yo + q] = bidx[q];
    }
  }
}

// gather backward: dx[n][h][w][c] = sum over windows covering (h,w)
template <int VEC>
__global__ void pool_bwd_kernel(const uint16_t* dy, const int* argmax,
                                uint16_t* dx, int N, int H, int W, int C,
                                int OH, int OW, int ky, int kx, int sy, int sx,
                                int pt, int pl, int mode, const uint16_t* aux,
                                int aux_act) {
  const int CV = C / VEC;
  long long total = (long long)N * H * W * CV;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int cv = (int)(e % CV);
    long long pix = e / CV;
    int w = (int)(pix % W);
    long long t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    long long xoff = pix * C + cv * VEC;
    // windows oh with oh*sy - pt <= h < oh*sy - pt + ky
    int hp = h + pt, wp = w + pl;
    int oh0 = hp - ky + 1 <= 0 ? 0 : (hp - ky + sy) / sy;
    int oh1 = min(OH - 1, hp / sy);
    int ow0 = wp - kx + 1 <= 0 ? 0 : (wp - kx + sx) / sx;
    int ow1 = min(OW - 1, wp / sx);
    float acc[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        long long yo = (((long long)n * OH + oh) * OW + ow) * C + cv * VEC;
        uint16_t g[VEC];
        if (VEC == 8) *(uint4*)g = *(const uint4*)(dy + yo);
        else g[0] = dy[yo];
        if (mode == POOL_AVG) {
          int hh0 = max(oh * sy - pt, 0), hh1 = min(oh * sy - pt + ky, H);
          int ww0 = max(ow * sx - pl, 0), ww1 = min(ow * sx - pl + kx, W);
          float inv = 1.f / (float)max((hh1 - hh0) * (ww1 - ww0), 1);
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[q] += bf2f(g[q]) * inv;
        } else {
#pragma unroll
          for (int q = 0; q < VEC; ++q)
            if (argmax[yo + q] == (int)(xoff + q)) acc[q] += bf2f(g[q]);
        }
      }
    uint16_t o[VEC];
    if (aux) {
      uint16_t a[VEC];
      if (VEC == 8) *(uint4*)a = *(const uint4*)(aux + xoff);
      else a[0] = aux[xoff];
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[q] *= act_bwd(bf2f(a[q]), aux_act);
    }
#pragma unroll
    for (int q = 0; q < VEC; ++q) o[q] = f2bf(acc[q]);
    if (VEC == 8) *(uint4*)(dx + xoff) = *(uint4*)o;
    else dx[xoff] = o[0];
  }
}

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
      y[p * C + c] = f2bf(xs[c] * exp2f(-beta * log2f(s)));
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
    int idx = 0;
    for (int c = lane; c < C; c += 64, ++idx) {
      float s = 0.f;
      int c0 = max(0, c - half), c1 = min(C - 1, c + half);
      for (int j = c0; j <= c1; ++j) s += xs[j] * xs[j];
      s = k + alpha * s;
      float sb = exp2f(-beta * log2f(s));
      float g = bf2f(dy[p * C + c]);
      ts[c] = g * xs[c] * sb / s;
      keep[idx] = g * sb;
    }
    __builtin_amdgcn_wave_barrier();
    idx = 0;
    for (int c = lane; c < C; c += 64, ++idx) {
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
}  // namespace

HVK_API int hvk_pool_fwd(const void* x, void* y, int* argmax, int N, int H,
                         int W, int C, int OH, int OW, int ky, int kx, int sy,
                         int sx, int pt, int pl, int mode, hipStream_t s) {
  if (C % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    long long total = (long long)N * OH * OW * (C / 8);
    hipLaunchKernelGGL(pool_fwd_kernel<8>, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode);
  } else {
    long long total = (long long)N * OH * OW * C;
    hipLaunchKernelGGL(pool_fwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)x, (uint16_t*)y, argmax, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode);
  }
  return (int)hipGetLastError();
}

HVK_API int hvk_pool_bwd(const void* dy, const int* argmax, void* dx, int N,
                         int H, int W, int C, int OH, int OW, int ky, int kx,
                         int sy, int sx, int pt, int pl, int mode,
                         const void* aux, int aux_act, hipStream_t s) {
  if (C % 8 == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0 &&
      ((uintptr_t)aux & 15) == 0) {
    long long total = (long long)N * H * W * (C / 8);
    hipLaunchKernelGGL(pool_bwd_kernel<8>, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, (const uint16_t*)aux,
                       aux_act);
  } else {
    long long total = (long long)N * H * W * C;
    hipLaunchKernelGGL(pool_bwd_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s,
                       (const uint16_t*)dy, argmax, (uint16_t*)dx, N, H, W, C, OH,
                       OW, ky, kx, sy, sx, pt, pl, mode, (const uint16_t*)aux,
                       aux_act);
  }
  return (int)hipGetLastError();
}

HVK_API int hvk_lrn_fwd(const void* x, void* y, long long P, int C, int n,
                        float alpha, float beta, float k, hipStream_t s) {
  if (C > 1024) return -1;
  hipLaunchKernelGGL(lrn_fwd_kernel, dim3(grid_for(P, 4)), dim3(256), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, P, C, n, alpha, beta, k);
  return (int)hipGetLastError();
}

HVK_API int hvk_lrn_bwd(const void* x, const void* dy, void* dx, long long P,
                        int C, int n, float alpha, float beta, float k,
                        const void* aux, int aux_act, hipStream_t s) {
  if (C > 1024) return -1;
  hipLaunchKernelGGL(lrn_bwd_kernel, dim3(grid_for(P, 4)), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)dy, (uint16_t*)dx, P,
                     C, n, alpha, beta, k, (const uint16_t*)aux, aux_act);
  return (int)hipGetLastError();
}
