// wgrad_fp8.hip - fp8 convolution weight gradient on the f8f6f4 matrix core:
//   dW[oc][kh][kw][c] += sum_p dY8[p][oc] * im2col(X8)[p][kk] / (s_dY s_X)
// with dY8 the e5m2 gradient copy and X8 the e4m3 input copy the fp8 forward
// / backward-data already hold (docs/OPS.md §FP8).  This completes the fp8
// layer: forward, backward-data and weight gradient all run on
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 rate per clock).
//
// Both operands are MN-major (the reduction runs over pixels p, the slow
// index of both NHWC tensors), so they are staged as [128 pixels][128 B]
// LDS images and read TRANSPOSED into the MFMA's K-major lane layout with
// ds_read_b64_tr_b8: per 16-lane group it reads a block of 8 rows x 16 byte
// columns and hands lane i column i's 8 bytes (row q in byte q) - measured
// on gfx950 with tools/probes/ds_read_tr8.hip.  Four such reads give a lane
// its 32 consecutive pixels of one column (lane l: column l & 15, pixels
// 32 (l >> 4) ... +31, the f8f6f4 operand map of gemm_fp8.hip).
//
// LDS image swizzle: 16-B chunk c of image row r is stored at c ^ f(r),
// f(r) = ((r >> 1) & 3) | ((r >> 5) & 1) << 2, so the 32 lanes of a
// half-wave (two 16-lane groups = rows 32g + 8j .. +7 and 32(g+1) + 8j ..,
// one 16-B chunk each) cover all 64 banks once.  The LDS-DMA writes lane-
// linear, so the permutation is applied to the SOURCE chunk (rule 21 of
// cdna_hip_programming.md §5.4).
//
// Tile 128 (oc) x 128 (kk) x 128 (pixels), 8 waves (2 x 4, each 64 x 32),
// double-buffered LDS-DMA (buffer descriptors, out-of-range -> zeros) with
// the next tile in flight across the barrier; split over pixels, f32
// atomics into the gradient (the bf16 weight-gradient scheme).  The bias
// gradient rides along as four MFMAs against an all-ones operand.
#include "fp8_common.h"
#include "conv_geom.h"

using namespace hvk;

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) int i32x2;

namespace {

constexpr int TM = 128, TN = 128, TK = 128, NT = 512;
constexpr int IMG = TK * 128;  // bytes per operand image (one stage)

__device__ __forceinline__ int swz(int r) {
  return ((r >> 1) & 3) | (((r >> 5) & 1) << 2);
}

struct WgradGeom8 {
  ConvGeom g;
  int P, KK;   // pixels (N*OH*OW), kk per group (KH*KW*Cg)
};

template <int FA, int FB>
__global__ void __launch_bounds__(NT, 2)
wgrad_fp8_kernel(const uint8_t* __restrict__ dy8, const uint8_t* __restrict__ x8,
                 float* __restrict__ dw, float* __restrict__ dbias,
                 WgradGeom8 wg, int k_split, int tiles_n, int tiles,
                 int splits, const float* sdy, const float* sx, int hist,
                 float fmax_dy, float fmax_x) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[4 * IMG];
  const ConvGeom& g = wg.g;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gs = wgid / tiles;
  const int gi = gs / splits;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int kbeg = (gs - gi * splits) * k_split;
  const int kend = min(wg.P, kbeg + k_split);
  if (kbeg >= kend) return;
  const int m0 = tm * TM, n0 = tn * TN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;   // wave tile 64 (oc) x 32 (kk)
  const int fr = lane & 15, fg = lane >> 4;

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias gradient: the first column tile's wn == 0 waves also multiply their
  // dY8 fragments by an all-ones B operand (exact 1.0 in B's format), so
  // bias[oc] = sum_p dY8[p][oc] / s_dY comes out of 4 more MFMAs per K tile
  const bool do_bias = dbias != nullptr && tn == 0 && wn == 0;
  f32x4 accb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int one8 = FB == 0 ? 0x38383838 : 0x3C3C3C3C;
  const i32x8 ones = {one8, one8, one8, one8, one8, one8, one8, one8};

  // ---- DMA slots: image rows 8I .. 8I+7 (I = 2w + i), lane -> row
  // 8I + (lane >> 3), physical chunk lane & 7 = logical chunk ^ swz(row)
  const __amdgpu_buffer_rsrc_t ra = dma_rsrc(dy8);
  const __amdgpu_buffer_rsrc_t rb = dma_rsrc(x8);
  int arow[2], acol[2];      // A: image row, oc of the chunk (or -1)
  int bkh[2], bkw[2], bch[2], bok[2];
  int rowi[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int I = 2 * w + i;
    const int row = 8 * I + (lane >> 3);
    const int c = (lane & 7) ^ swz(row);
    rowi[i] = row;
    arow[i] = row;
    const int oc = m0 + 16 * c;
    acol[i] = oc < g.OCg ? gi * g.OCg + oc : -1;
    const int kk = n0 + 16 * c;
    bok[i] = kk < wg.KK;
    uint32_t tp, ch, kh, kw;
    fdivmod(bok[i] ? kk : 0, g.fCg, tp, ch);
    fdivmod(tp, g.fKW, kh, kw);
    bkh[i] = (int)kh - g.pt;
    bkw[i] = (int)kw - g.pl;
    bch[i] = gi * g.Cg + (int)ch;
  }
  auto issue = [&](int k0, uint8_t* sA, uint8_t* sB) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = k0 + rowi[i];
      const bool pin = p < kend;
      // A: dY8[p][oc .. oc + 15]
      const uint32_t va = (pin & (acol[i] >= 0))
                              ? (uint32_t)p * (uint32_t)g.OC + (uint32_t)acol[i]
                              : kBufOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)(sA + (2 * w + i) * 1024),
          16, va, 0, 0, 0);
      // B: X8[n][oh*sy + kh][ow*sx + kw][ch .. ch + 15]
      uint32_t n, rem, oh, ow;
      fdivmod((uint32_t)(pin ? p : 0), g.fOHOW, n, rem);
      fdivmod(rem, g.fOW, oh, ow);
      const int ih = (int)oh * g.sy + bkh[i], iw = (int)ow * g.sx + bkw[i];
      const bool ok = pin & (bok[i] != 0) & ((unsigned)ih < (unsigned)g.H) &
                      ((unsigned)iw < (unsigned)g.W);
      const uint32_t vb =
          ok ? (uint32_t)((((int)n * g.H + ih) * g.W + iw) * g.C + bch[i])
             : kBufOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(sB + (2 * w + i) * 1024),
          16, vb, 0, 0, 0);
    }
  };
  // operand of MFMA column block `col0` (16 columns): lane l gets column
  // col0 + (l & 15), pixels 32 (l >> 4) .. +31 - four transposed reads;
  // lane 2q + p of each 16-lane group supplies row q's 8 bytes at column
  // col0 + 8p
  const int q = fr >> 1, pp = fr & 1;
  auto frag = [&](const uint8_t* s, int col0) -> i32x8 {
    i32x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 32 * fg + 8 * j + q;
      const int c = col0 >> 4;
      const uint8_t* a = s + r * 128 + ((c ^ swz(r)) << 4) + 8 * pp;
      const i32x2 h = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
          (__attribute__((address_space(3))) i32x2*)a);
      v[2 * j] = h[0];
      v[2 * j + 1] = h[1];
    }
    return v;
  };
  auto compute = [&](const uint8_t* sA, const uint8_t* sB) {
    i32x8 af[4], bfv[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(sA, wm * 64 + i * 16);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfv[j] = frag(sB, wn * 32 + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            af[i], bfv[j], acc[i][j], FA, FB, 0, 127, 0, 127);
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        accb[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            af[i], ones, accb[i], FA, FB, 0, 127, 0, 127);
    }
  };

  const int nk = (kend - kbeg + TK - 1) / TK;
  issue(kbeg, smem, smem + 2 * IMG);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue(kbeg + (kt + 1) * TK, smem + (cur ^ 1) * IMG,
            smem + 2 * IMG + (cur ^ 1) * IMG);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // next tile in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(smem + cur * IMG, smem + 2 * IMG + cur * IMG);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // dequantise (1 / (s_dY s_X)) and add: accumulator (i, j)[rr] is
  // dW row m0 + 64 wm + 16 i + 4 fg + rr, column n0 + 32 wn + 16 j + fr
  const float sdv = fp8_scale(sdy, hist, fmax_dy);
  const float alpha = 1.f / (sdv * fp8_scale(sx, hist, fmax_x));
  if (do_bias && fr == 0) {
    // every column of accb holds the row sums: lanes of column 0 add them
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = m0 + wm * 64 + i * 16 + fg * 4 + rr;
        if (m < g.OCg) atomicAdd(dbias + gi * g.OCg + m, accb[i][rr] / sdv);
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + fr;
      if (n >= wg.KK) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = m0 + wm * 64 + i * 16 + fg * 4 + rr;
        if (m < g.OCg)
          atomicAdd(dw + (long long)(gi * g.OCg + m) * wg.KK + n,
                    acc[i][j][rr] * alpha);
      }
    }
}

}  // namespace

// dW (f32, [OC][KH][KW][C/g]) += conv weight gradient from the fp8 copies
// dY8 (NHWC, format fdy) and X8 (NHWC, format fx); OC/g, C/g, C and OC
// multiples of 16, both tensors < 2 GiB.  splits: pixel splits (f32
// atomics).  dB (optional, f32 [OC]) += sum over pixels of dY8 / s_dY.
HVK_API int hvk_conv_wgrad_fp8(const void* X8, const void* dY8, float* dW,
                               float* dB,
                               int N, int H, int W, int C, int OC, int KH,
                               int KW, int sy, int sx, int pt, int pl, int OH,
                               int OW, int groups, int splits, int fx,
                               int fdy, const float* sxs, const float* sdys,
                               int hist, float fmax_x, float fmax_dy,
                               hipStream_t s) {
  WgradGeom8 wg;
  wg.g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  wg.P = N * OH * OW;
  wg.KK = KH * KW * wg.g.Cg;
  const ConvGeom& g = wg.g;
  if ((g.Cg & 15) || (g.OCg & 15) || (C & 15) || (OC & 15) || !al16(X8) ||
      !al16(dY8))
    return -3;
  if ((long long)N * H * W * C >= kBufMaxBytes ||
      (long long)wg.P * OC >= kBufMaxBytes)
    return -3;
  if (fx != 0 && fx != 1) return -2;
  if (splits < 1) splits = 1;
  int k_split = (wg.P + splits - 1) / splits;
  k_split = (k_split + TK - 1) / TK * TK;
  splits = (wg.P + k_split - 1) / k_split;
  const int tiles_m = (g.OCg + TM - 1) / TM, tiles_n = (wg.KK + TN - 1) / TN;
  const int tiles = tiles_m * tiles_n;
  dim3 grid((unsigned)((long long)tiles * splits * groups));
  // A = dY8 (cbsz = its format), B = X8 (blgp)
#define HVK_WG8(FA, FB)                                                       \
  hipLaunchKernelGGL((wgrad_fp8_kernel<FA, FB>), grid, dim3(NT), 0, s,         \
                     (const uint8_t*)dY8, (const uint8_t*)X8, dW, dB, wg,      \
                     k_split, tiles_n, tiles, splits, sdys, sxs, hist,         \
                     fmax_dy, fmax_x)
  if (fdy == 1 && fx == 0) HVK_WG8(1, 0);
  else if (fdy == 0 && fx == 0) HVK_WG8(0, 0);
  else if (fdy == 1 && fx == 1) HVK_WG8(1, 1);
  else HVK_WG8(0, 1);
#undef HVK_WG8
  return (int)launch_status(s);
}
