// conv_hc.hip - stride-1 convolution forward / backward-data with a
// channel-chunked input window shared by every tap ("halo, chunked").
//
//   Y[p][oc] = act(sum_{c, kh, kw} X[n(p)][oh(p)+kh-pt][ow(p)+kw-pl][c] *
//                                  W[oc][kh][kw][c] + bias[oc])
//
// Why (round 5, VERDICT r4 "next" #2): the implicit GEMM (gemm_core.h, T4)
// gathers im2col(X) - KH*KW shifted copies of the same pixels - through
// LDS-DMA for every K step, and the DMA pieces, not the MFMAs, bound those
// loops (profiles/r4/t4_ablation/README.md: without the main-loop DMA
// +35-40 % on the convolutions).  conv_halo.hip holds a whole-channel halo
// of a 128-pixel tile and streams the weights, which caps its tile at 128
// pixels and leaves ~1/128 B/FLOP of weight traffic.  Here one workgroup of
// eight waves owns a TPX (256 | 512) pixel x BN output-channel tile and
// walks the source channels of its group in chunks of 16; per chunk (one K
// stage) it DMAs
//   * the WINDOW of the tile: the image rows its pixels span plus the kh
//     halo, all columns plus the kw halo, 16 channels (32-B slots), and
//   * the weights of the chunk: BN rows x every tap x 16 channels,
// and every tap reads its A fragments out of the same window at a constant
// slot offset kh * Wp + kw.  Per stage the MFMAs cover BN x TPX x taps x 16
// MACs: for 3 x 3 at 256 x 128 ~0.005 operand bytes per FLOP, against 0.013
// for the T4 loop.
//
// K order inside a stage: each 16x16x32 MFMA takes TWO taps x 16 channels
// (k-groups 0-1 the first tap's halves, 2-3 the second's); an odd tap count
// pads the last MFMA with a zero-weight tap.  Weight rows in LDS are
// TP = 2 * ceil(T / 2) + 1 (odd) 32-B granules apart, so the 16 rows of a
// ds_read_b128 lane group hit 16 distinct bank groups; the window's slot
// row pitch Wp = OW + 8 keeps 8 consecutive output pixels on slots distinct
// mod 8 across row wraps (the A reads' conflict-free shape; only the one
// fragment per image that straddles two images conflicts).
//
// Window layout (full rows, any number of images): window row r of a tile
// starting at output row oh0 of image n0 is padded row oh0 + r of image n0
// while r < rc = OH - oh0 + KH - 1, then padded row (r - rc) % HPd of image
// n0 + 1 + (r - rc) / HPd (HPd = OH + KH - 1: each image contributes its
// rows plus the kh halo, so images never share a slot).  Padded row q is
// source row q - pt; zeros outside the image come from the buffer
// descriptor's out-of-range fill.
//
// Persistent: one workgroup per CU walks (pixel tile, group, n-tile) items;
// the (item, chunk) sequence is one double-buffered pipeline, so the next
// item's first chunk is in flight while the current item's last chunk runs,
// and each item's epilogue (bias, activation, derivative of the layer
// below, bf16 8-B stores straight from the accumulators) overlaps the
// following chunk's DMA.
//
// Backward-data (stride 1) is the same kernel: dX = conv(dY, W'), W' the
// flipped, transposed filter bank read from the dgrad permutation
// wt[g][c][kh][kw][oc] at tap T - 1 - t, window origin KH-1-pt / KW-1-pl.
//
// Reference counterpart: Znicz conv forward / backward-data
// (/root/reference/ocl/matrix_multiplication_precise.cl:47-185 through the
// conv units' im2col); SURVEY §7.4 item 2.
#include <algorithm>
#include <numeric>

#include "conv_geom.h"

// diagnostic builds only (wrong results by design): 1 no DMA, 2 no epilogue
// stores, 4 no MFMAs
#ifndef HVK_HC_ABL
#define HVK_HC_ABL 0
#endif

using namespace hvk;

namespace {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;

struct HcGeom {
  int N, H, W, C;     // window source (x or dY), NHWC, C channels in total
  int OH, OW;         // output pixels per image
  int OCT, OCg;       // output channels: total, per group
  int CG;             // source channels per group (multiple of 16)
  int pt, pl;         // source row = oh + kh - pt, column = ow + kw - pl
  int P, OHW;         // N * OH * OW, OH * OW
  int Wp, HPd, WIN;   // slot row pitch, padded rows per image, window bytes
  int NT, G, items;   // n-tiles per group, groups, (tile, group, n-tile) items
  int flip;           // backward-data: weight tap T - 1 - t
  FastDiv fOW, fOHW, fHPd, fWp;
};

// KH x KW taps; WM x WN = 8 waves, each 64 pixels x NJW * 16 channels;
// NBW: window DMA pieces per wave (upper bound, the plan checks)
template <int KH, int KW, int WM, int WN, int NJW, int NBW>
__global__ void __launch_bounds__(512, 1)
conv_hc_kernel(const uint16_t* __restrict__ src,
               const uint16_t* __restrict__ wts, const float* __restrict__ bias,
               uint16_t* __restrict__ out, const uint16_t* __restrict__ aux,
               int act, int aux_act, HcGeom g) {
  constexpr int T = KH * KW;
  constexpr int NKS = (T + 1) / 2;           // MFMA k-steps per chunk
  constexpr int TP = 2 * NKS + 1;            // granules per weight row (odd)
  constexpr int NWV = WM * WN;
  static_assert(NWV == 8, "eight waves");
  constexpr int MI = 4;                      // 64 pixels per wave
  constexpr int TPX = WM * 64;
  constexpr int BN = WN * NJW * 16;
  constexpr int WB = BN * TP * 32;           // weight bytes per stage
  constexpr int NWP = (WB + 1023) / 1024;    // weight DMA pieces
  constexpr int NWW = (NWP + NWV - 1) / NWV;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  lds_u8* sm = (lds_u8*)smem;
  const uint32_t STAGE = (uint32_t)g.WIN + NWP * 1024;
  const int NBP = g.WIN >> 10;               // window pieces per stage
  const int NC = g.CG >> 4;                  // chunks (K stages) per item
  const int KT = T * g.CG;                   // weight row length (elements)

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w % WM, wn = w / WM;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- weight DMA: this lane's 16-B chunk of each of its pieces ->
  // (row n, granule tp, half); pad granules and rows read zeros
  uint32_t wq[NWW];
#pragma unroll
  for (int i = 0; i < NWW; ++i) {
    const int pi = w + NWV * i;
    const int ib = pi * 1024 + 16 * lane;
    const int n = ib / (TP * 32);
    const int rem = ib - n * (TP * 32);
    const int tp = rem >> 5, half = (rem >> 4) & 1;
    const bool ok = pi < NWP && n < BN && tp < T;
    const int tap = g.flip ? T - 1 - tp : tp;
    wq[i] = ok ? (uint32_t)(n * KT + tap * g.CG + half * 8) * 2u : kBufOOB;
  }
  // ---- window DMA: (window row, column, half) of this lane's chunks
  uint32_t pw[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int pi = w + NWV * i;
    const uint32_t slot = (uint32_t)(pi * 1024 + 16 * lane) >> 5;
    const uint32_t r = fdiv(slot, g.fWp);
    const uint32_t cs = slot - r * (uint32_t)g.Wp;
    const bool ok = pi < NBP && (int)cs < g.OW + KW - 1;
    pw[i] = r | (cs << 10) | ((uint32_t)(lane & 1) << 30) |
            (ok ? 0x80000000u : 0u);
  }
  // ---- A fragment tap offsets per k-step (k-group fq: tap 2s + fq / 2,
  // channel half fq % 2); the pad tap reads tap 0 (finite, zero weight)
  uint32_t ofs[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    int tp = 2 * s + (fq >> 1);
    if (tp >= T) tp = 0;
    const int kh = tp / KW, kw = tp - (tp / KW) * KW;
    ofs[s] = (uint32_t)((kh * g.Wp + kw) * 32 + (fq & 1) * 16);
  }
  // ---- B fragment row bases (weights: row n, k-group fq)
  uint32_t bq[NJW];
#pragma unroll
  for (int j = 0; j < NJW; ++j)
    bq[j] = (uint32_t)(((wn * NJW + j) * 16 + fr) * (TP * 32) + fq * 16);

  const __amdgpu_buffer_rsrc_t rs = dma_rsrc(src);
  const __amdgpu_buffer_rsrc_t rw = dma_rsrc(wts);
  const uint32_t rowbytes = (uint32_t)g.W * g.C * 2u;
  const uint32_t pixbytes = (uint32_t)g.C * 2u;

  // item -> (pixel tile, group, n-tile), n-tile fastest
  auto decode = [&](int it, int& ptl, int& gi, int& nt) {
    nt = it % g.NT;
    const int r = it / g.NT;
    gi = r % g.G;
    ptl = r / g.G;
  };
  auto issue = [&](int it, int c, uint32_t stb) {
    if constexpr ((HVK_HC_ABL & 1) != 0) return;
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
    const uint32_t n0 = fdiv(p0, g.fOHW);
    const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
    const int rc = g.OH - (int)oh0 + KH - 1;
    const uint32_t cofs = (uint32_t)(gi * g.CG + c * 16) * 2u;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (w + NWV * i < NBP) {   // wave-uniform
        const int r = (int)(pw[i] & 1023u);
        const int cs = (int)((pw[i] >> 10) & 0xfffffu);
        int j, lr;
        if (r < rc) {
          j = 0;
          lr = (int)oh0 + r;
        } else {
          const int q = (int)fdiv((uint32_t)(r - rc), g.fHPd);
          j = 1 + q;
          lr = r - rc - q * g.HPd;
        }
        const int ih = lr - g.pt, iw = cs - g.pl;
        const uint32_t n = n0 + (uint32_t)j;
        const bool ok = (pw[i] >> 31) && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W && n < (uint32_t)g.N;
        const uint32_t v = ok ? (n * (uint32_t)g.H + (uint32_t)ih) * rowbytes +
                                    (uint32_t)iw * pixbytes + cofs +
                                    ((pw[i] >> 30) & 1u) * 16u
                              : kBufOOB;
        dma16(rs, smem + stb + (w + NWV * i) * 1024, v);
      }
    }
    const uint32_t wofs =
        ((uint32_t)(gi * g.OCg + nt * BN) * (uint32_t)KT + c * 16) * 2u;
#pragma unroll
    for (int i = 0; i < NWW; ++i) {
      if (w + NWV * i < NWP)   // wave-uniform
        dma16(rw, smem + stb + g.WIN + (w + NWV * i) * 1024,
              wq[i] >= kBufOOB ? kBufOOB : wq[i] + wofs);
    }
  };
  // window slot bytes of this lane's pixels (fr of each m-tile)
  uint32_t bb[MI];
  auto slots = [&](int it) {
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
    const uint32_t n0 = fdiv(p0, g.fOHW);
    const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
    const int rc = g.OH - (int)oh0 + KH - 1;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const uint32_t p = p0 + wm * 64 + i * 16 + fr;
      if (p >= (uint32_t)g.P) {   // past the last pixel: slot 0 (finite)
        bb[i] = 0;
        continue;
      }
      const uint32_t n = fdiv(p, g.fOHW);
      const uint32_t pin = p - n * (uint32_t)g.OHW;
      const uint32_t oh = fdiv(pin, g.fOW);
      const int ow = (int)(pin - oh * (uint32_t)g.OW);
      const int j = (int)(n - n0);
      const int row = j == 0 ? (int)(oh - oh0) : rc + (j - 1) * g.HPd + (int)oh;
      bb[i] = (uint32_t)(row * g.Wp + ow) * 32u;
    }
  };

  const int nwg = gridDim.x;
  int item = xcd_remap(blockIdx.x, nwg);
  if (item >= g.items) return;
  issue(item, 0, 0);
  slots(item);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  f32x4 acc[MI][NJW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int c = 0;
  uint32_t cur = 0;
  for (;;) {
    int nitem = item, nc = c + 1;
    if (nc == NC) {
      nc = 0;
      nitem += nwg;
    }
    const bool more = nitem < g.items;
    if (more) issue(nitem, nc, cur ^ STAGE);
    const uint32_t wb = cur + (uint32_t)g.WIN;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      bf16x8 a[MI], b[NJW];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[i] = *(lds_bf16x8*)(sm + cur + bb[i] + ofs[s]);
#pragma unroll
      for (int j = 0; j < NJW; ++j)
        b[j] = *(lds_bf16x8*)(sm + wb + bq[j] + s * 64);
      if constexpr ((HVK_HC_ABL & 4) == 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                b[j], a[i], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          acc[i][0][0] += (float)a[i][0] + (float)b[0][0];
      }
    }
    // the next chunk landed; every read of this one done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c == NC - 1) {
      // epilogue (lane: D[n = fq * 4 + r][m = fr], 4 consecutive output
      // channels of one pixel): bias, activation, derivative of the layer
      // below, bf16, one 8-B store per (m-tile, n-tile)
      int ptl, gi, nt;
      decode(item, ptl, gi, nt);
      const uint32_t p0 = (uint32_t)ptl * TPX;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const uint32_t p = p0 + wm * 64 + i * 16 + fr;
        if (p >= (uint32_t)g.P ||
            ((HVK_HC_ABL & 2) && acc[i][0][0] != 1234.5f))
          continue;
#pragma unroll
        for (int j = 0; j < NJW; ++j) {
          const int oc = gi * g.OCg + nt * BN + (wn * NJW + j) * 16 + fq * 4;
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2],
                        acc[i][j][3]};
          if (bias) {
            const float4 bv = *(const float4*)(bias + oc);
            v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
          }
          act_fwd_n<4>(v, act);
          const long long oi = (long long)p * g.OCT + oc;
          if (aux) {
            const uint2 av = *(const uint2*)(aux + oi);
            const float y[4] = {__uint_as_float(av.x << 16),
                                __uint_as_float(av.x & 0xffff0000u),
                                __uint_as_float(av.y << 16),
                                __uint_as_float(av.y & 0xffff0000u)};
            act_bwd_mul_n<4>(v, y, aux_act);
          }
          *(uint2*)(out + oi) = make_uint2(pack_bf16x2(v[0], v[1]),
                                           pack_bf16x2(v[2], v[3]));
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (more) slots(nitem);
    }
    if (!more) break;
    item = nitem;
    c = nc;
    cur ^= STAGE;
  }
}

struct HcPlan {
  int var;      // 0: not taken
  size_t lds;
  int grid;
  HcGeom g;
};

constexpr int kCUs = 256;
constexpr int kNBW = 8;   // window pieces per wave: 64 KiB windows at most
int g_hc_variant = -1;    // -1 automatic, 0 off, > 0 forced configuration

struct HcCand { int var, KH, KW, WM, WN, NJW; };
// per kernel size, in order of preference (the first whose n-tile divides
// the group's outputs and whose two stages fit the LDS)
constexpr HcCand kHcCands[] = {
    {1, 3, 3, 4, 2, 4},   // 256 px x 128 ch: AlexNet conv3 / conv5 fwd, conv3 dgrad
    {2, 3, 3, 4, 2, 3},   // 256 px x 96 ch: conv1 (s2d), conv4 fwd, conv4 / 5 dgrad
    {3, 3, 3, 8, 1, 4},   // 512 px x 64 ch: VGG-16 64-channel layers
    {4, 5, 5, 4, 2, 2},   // 256 px x 64 ch: AlexNet conv2 fwd
    {5, 5, 5, 8, 1, 3},   // 512 px x 48 ch: AlexNet conv2 dgrad
};

int hc_nbytes_w(const HcCand& k) {
  const int T = k.KH * k.KW, TP = 2 * ((T + 1) / 2) + 1;
  const int BN = k.WN * k.NJW * 16;
  return (BN * TP * 32 + 1023) / 1024 * 1024;
}

HcPlan hc_plan(int N, int H, int W, int C, int OH, int OW, int OCT, int KH,
               int KW, int pt, int pl, int groups, bool flip) {
  HcPlan p{};
  HcGeom& g = p.g;
  if (g_hc_variant == 0) return p;
  const int CG = C / groups, OCg = OCT / groups;
  if (CG % 16 || OCg % 16 || OCT % 4) return p;
  if ((long long)N * H * W * C * 2 >= kBufMaxBytes) return p;
  if ((long long)N * OH * OW >= (1ll << 31)) return p;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.OCT = OCT;
  g.OCg = OCg; g.CG = CG; g.pt = pt; g.pl = pl; g.G = groups;
  g.P = N * OH * OW;
  g.OHW = OH * OW;
  g.Wp = OW + 8;
  g.HPd = OH + KH - 1;
  g.flip = flip ? 1 : 0;
  if (OW + KW - 1 > g.Wp || g.Wp >= (1 << 20)) return p;
  for (const HcCand& k : kHcCands) {
    if (k.KH != KH || k.KW != KW) continue;
    if (g_hc_variant > 0 && k.var != g_hc_variant) continue;
    const int BN = k.WN * k.NJW * 16, TPX = k.WM * 64;
    if (OCg % BN) continue;
    // window rows: the most any tile needs (the pattern of tile starts
    // repeats with the image, so one period of starts covers every tile)
    const long long tiles = ((long long)g.P + TPX - 1) / TPX;
    const long long per = g.OHW / std::gcd(TPX, g.OHW);
    const long long nt = tiles < per ? tiles : per;
    int wr = 0;
    for (long long tl = 0; tl < nt; ++tl) {
      const long long p0 = tl * TPX, p1 = std::min<long long>(p0 + TPX,
                                                              g.P) - 1;
      const int n0 = (int)(p0 / g.OHW), oh0 = (int)(p0 % g.OHW) / OW;
      const int n1 = (int)(p1 / g.OHW), oh1 = (int)(p1 % g.OHW) / OW;
      const int rc = OH - oh0 + KH - 1;
      const int j = n1 - n0;
      const int row = j == 0 ? oh1 - oh0 : rc + (j - 1) * g.HPd + oh1;
      wr = std::max(wr, row + KH);
    }
    if (wr >= 1024) continue;
    g.WIN = (wr * g.Wp * 32 + 1023) / 1024 * 1024;
    if (g.WIN / 1024 > 8 * kNBW) continue;
    const size_t lds = 2 * (size_t)(g.WIN + hc_nbytes_w(k));
    if (lds > 160 * 1024) continue;
    g.NT = OCg / BN;
    g.items = (int)(tiles * groups * g.NT);
    g.fOW = make_fastdiv(OW);
    g.fOHW = make_fastdiv(g.OHW);
    g.fHPd = make_fastdiv(g.HPd);
    g.fWp = make_fastdiv(g.Wp);
    p.lds = lds;
    p.grid = std::min(g.items, kCUs);
    p.var = k.var;
    return p;
  }
  return p;
}

template <int KH, int KW, int WM, int WN, int NJW>
hipError_t go_hc(const HcPlan& p, const void* src, const void* wts,
                 const float* bias, void* out, const void* aux, int act,
                 int aux_act, hipStream_t s) {
  auto kern = conv_hc_kernel<KH, KW, WM, WN, NJW, kNBW>;
  static bool attr = false;   // once per instantiation, before any capture
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(
        (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
        160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)p.grid), dim3(512), p.lds, s,
                     (const uint16_t*)src, (const uint16_t*)wts, bias,
                     (uint16_t*)out, (const uint16_t*)aux, act, aux_act, p.g);
  return launch_status(s);
}

hipError_t hc_launch(const HcPlan& p, const void* src, const void* wts,
                     const float* bias, void* out, const void* aux, int act,
                     int aux_act, hipStream_t s) {
  switch (p.var) {
    case 1: return go_hc<3, 3, 4, 2, 4>(p, src, wts, bias, out, aux, act,
                                        aux_act, s);
    case 2: return go_hc<3, 3, 4, 2, 3>(p, src, wts, bias, out, aux, act,
                                        aux_act, s);
    case 3: return go_hc<3, 3, 8, 1, 4>(p, src, wts, bias, out, aux, act,
                                        aux_act, s);
    case 4: return go_hc<5, 5, 4, 2, 2>(p, src, wts, bias, out, aux, act,
                                        aux_act, s);
    case 5: return go_hc<5, 5, 8, 1, 3>(p, src, wts, bias, out, aux, act,
                                        aux_act, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Force a configuration (kHcCands var), 0 = off, -1 = automatic.
HVK_API void hvk_hc_variant(int v) { g_hc_variant = v; }

// Forward: Y[N][OH][OW][OC] = act(conv(X, W) + bias), stride 1, X bf16 NHWC,
// W [OC][KH][KW][C/g].  Returns 0, -2 when the shape does not take this
// kernel (the caller falls back), or a HIP error.
HVK_API int hvk_conv_fwd_hc(const void* X, const void* Wt, const float* bias,
                            void* Y, int N, int H, int W, int C, int OC,
                            int KH, int KW, int pt, int pl, int OH, int OW,
                            int groups, int act, hipStream_t s) {
  if (((uintptr_t)X & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)Y & 7) ||
      ((uintptr_t)bias & 15))
    return -2;
  HcPlan p = hc_plan(N, H, W, C, OH, OW, OC, KH, KW, pt, pl, groups, false);
  if (!p.var) return -2;
  return (int)hc_launch(p, X, Wt, bias, Y, nullptr, act, 0, s);
}

// Backward-data: dX[N][H][W][C] = conv^T(dY, W) [* act'(aux)], stride 1,
// from the dgrad weight permutation wt[g][c][kh][kw][oc].  -2: not taken.
HVK_API int hvk_conv_dgrad_hc(const void* dY, const void* Wt, void* dX, int N,
                              int H, int W, int C, int OC, int KH, int KW,
                              int pt, int pl, int OH, int OW, int groups,
                              const void* aux, int aux_act, hipStream_t s) {
  if (((uintptr_t)dY & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)dX & 7) ||
      ((uintptr_t)aux & 7))
    return -2;
  // the window source is dY (OH x OW, OC channels), the output dX (H x W, C
  // channels), origin KH - 1 - pt / KW - 1 - pl
  HcPlan p = hc_plan(N, OH, OW, OC, H, W, C, KH, KW, KH - 1 - pt,
                     KW - 1 - pl, groups, true);
  if (!p.var) return -2;
  return (int)hc_launch(p, dY, Wt, nullptr, dX, aux, 0, aux_act, s);
}
