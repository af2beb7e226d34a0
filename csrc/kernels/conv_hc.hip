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


using namespace hvk;

namespace {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

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
  int ts;             // conv_hc32: epilogue stores staged through LDS
  FastDiv fOW, fOHW, fHPd, fWp;
};

// KH x KW taps, KHS kh rows per K stage (a 5 x 5 splits into 3 + 2 rows:
// half the weights per stage, so a 512 x 64 tile fits two stages); WM x WN
// = 8 waves, each 64 pixels x NJW * 16 channels; NBW: window DMA pieces per
// wave (upper bound, the plan checks).
// ABL: diagnostic instantiations (compile-time so that the production loop
// carries no test): 1 no DMA after the first stage, 2 no epilogue stores,
// 4 no MFMAs, 8 no stage wait / barrier (wrong results by design); 16 / 32
// the DMA spread over the first third of the k-steps / issued at once, 64
// no software pipelining of the fragment reads (correct, for A/B runs), 256
// no weight DMA after the first stage (wrong results)
template <int KH, int KW, int KHS, int WM, int WN, int NJW, int NBW,
          int ABL = 0>
__global__ void __launch_bounds__(512, 1)
conv_hc_kernel(const uint16_t* __restrict__ src,
               const uint16_t* __restrict__ wts, const float* __restrict__ bias,
               uint16_t* __restrict__ out, const uint16_t* __restrict__ aux,
               int act, int aux_act, HcGeom g) {
  constexpr int T = KH * KW;
  constexpr int NH = (KH + KHS - 1) / KHS;   // stages per 16-channel chunk
  static_assert(NH <= 2, "at most two kh groups");
  // kh group h: rows h KHS .. + RH(h), T_h taps, NKS_h MFMA k-steps, TP_h
  // (odd) 32-B granules per weight row in LDS
  constexpr int RH0 = KHS, RH1 = KH - KHS;
  constexpr int T0 = RH0 * KW, T1 = RH1 * KW;
  constexpr int NKS0 = (T0 + 1) / 2, NKS1 = (T1 + 1) / 2;
  constexpr int TP0 = 2 * NKS0 + 1, TP1 = 2 * NKS1 + 1;
  constexpr int NWV = WM * WN;
  // eight waves (two per SIMD).  Four waves of 128 pixels (one per SIMD,
  // 512 registers, the accumulators in the AGPR half) measured 0.25-0.79x:
  // profiles/r5/ab_conv_hc_one_wave_per_simd_r5q.log
  static_assert(NWV == 8, "eight waves");
  constexpr int MI = 4;                      // 64 pixels per wave
  constexpr int WPX = MI * 16;
  constexpr int TPX = WM * WPX;
  constexpr int BN = WN * NJW * 16;
  constexpr int WB = BN * TP0 * 32;          // weight bytes per stage
  constexpr int NWP = (WB + 1023) / 1024;    // weight DMA pieces (at most)
  constexpr int NWW = (NWP + NWV - 1) / NWV;
  // n-tiles per store group: the weight rows are permuted so that a lane's
  // accumulators of NG consecutive n-tiles are 4 * NG consecutive output
  // channels (16- or 24-B stores, 16 * NG channels per pixel and group of 4
  // lanes; 128 B for NG 4) instead of 8-B pieces of 16-channel tiles
  // (two n-tiles per group for NJW 6 - 16-B stores - spilled inside the
  // k-loop and measured 10-12 % slower: profiles/r5/ablate_conv_hc_r5q.log)
  constexpr int NG = NJW % 4 == 0 ? 4 : NJW % 3 == 0 ? 3 : NJW % 2 == 0 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  lds_u8* sm = (lds_u8*)smem;
  // stage: window | weights | bias block (1 KiB: one DMA piece, the BN
  // output channels' bias of the item's last stage, wide tiles only)
  constexpr int BIASB = NJW <= 3 ? 0 : 1024;
  const uint32_t STAGE_B = (uint32_t)g.WIN + NWP * 1024;
  const uint32_t STAGE = STAGE_B + BIASB;
  const int NBP = g.WIN >> 10;               // window pieces per stage
  const int NQ = (g.CG >> 4) * NH;           // K stages per item
  const int KT = T * g.CG;                   // weight row length (elements)

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w % WM, wn = w / WM;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- weight DMA of kh group H: this lane's 16-B chunk of piece pi ->
  // byte offset in the filter bank (row n, granule tp, half), or kBufOOB
  // for pad granules and rows (recomputed per issue: registers, not time,
  // are short here)
  auto wq = [&](auto hc, int pi) __attribute__((always_inline)) -> uint32_t {
    constexpr int H = decltype(hc)::value;
    constexpr int TPH = H ? TP1 : TP0, TH = H ? T1 : T0;
    const int ib = pi * 1024 + 16 * lane;
    const int n = ib / (TPH * 32);
    const int rem = ib - n * (TPH * 32);
    const int tp = rem >> 5, half = (rem >> 4) & 1;
    const int tap0 = H * KHS * KW + tp;
    const int tap = g.flip ? T - 1 - tap0 : tap0;
    // LDS row n = 16 J + 4 f + r (n-tile J, lane group f) holds channel
    // 16 NG (J / NG) + 4 NG f + 4 (J % NG) + r
    const int J = n >> 4, f = (n >> 2) & 3, r = n & 3;
    const int ch = 16 * NG * (J / NG) + 4 * NG * f + 4 * (J % NG) + r;
    return (n < BN && tp < TH && pi * 1024 < BN * TPH * 32)
               ? (uint32_t)(ch * KT + tap * g.CG + half * 8) * 2u : kBufOOB;
  };
  // ---- A fragment tap offsets per k-step of each kh group (k-group fq:
  // tap 2s + fq / 2 of the group, channel half fq % 2); the pad tap reads
  // tap 0 (finite, zero weight).  Window rows of a stage start at its
  // group's first kh, so the offsets use the kh within the group
  uint32_t ofs0[NKS0], ofs1[NKS1 > 0 ? NKS1 : 1];
#pragma unroll
  for (int s = 0; s < NKS0; ++s) {
    int tp = 2 * s + (fq >> 1);
    if (tp >= T0) tp = 0;
    const int kh = tp / KW, kw = tp - (tp / KW) * KW;
    ofs0[s] = (uint32_t)((kh * g.Wp + kw) * 32 + (fq & 1) * 16);
  }
#pragma unroll
  for (int s = 0; s < NKS1; ++s) {
    int tp = 2 * s + (fq >> 1);
    if (tp >= T1) tp = 0;
    const int kh = tp / KW, kw = tp - (tp / KW) * KW;
    ofs1[s] = (uint32_t)((kh * g.Wp + kw) * 32 + (fq & 1) * 16);
  }

  const __amdgpu_buffer_rsrc_t rs = dma_rsrc(src);
  const __amdgpu_buffer_rsrc_t rw = dma_rsrc(wts);
  const uint32_t rowbytes = (uint32_t)g.W * g.C * 2u;
  const uint32_t pixbytes = (uint32_t)g.C * 2u;

  // item -> (pixel tile, group, n-tile), n-tile fastest
  auto decode = [&](int it, int& ptl, int& gi, int& nt)
                    __attribute__((always_inline)) {
    nt = it % g.NT;
    const int r = it / g.NT;
    gi = r % g.G;
    ptl = r / g.G;
  };
  // The DMA of one stage, prepared by prepare() and issued slot by slot:
  // per wave NBW window slots, NWW weight slots and one bias slot.
  // window source byte offsets of this lane's chunks (channel chunk 0; chunk
  // c adds 32 c) for the stage being loaded
  uint32_t pwb[NBW];
  uint32_t d_cofs = 0, d_wofs = 0, d_bofs = 0;
  int d_h = 0;
  bool d_bias = false;
  auto prepare = [&](int it, int q) __attribute__((always_inline)) {
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    const int c = q / NH, h = q - (q / NH) * NH;
    if (NH > 1 || c == 0) {   // wave-uniform: a new item or kh group
      const uint32_t p0 = (uint32_t)ptl * TPX;
      const uint32_t n0 = fdiv(p0, g.fOHW);
      const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
      const int rc = g.OH - (int)oh0 + KH - 1;
      const uint32_t gofs = (uint32_t)(gi * g.CG) * 2u;
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        // this lane's chunk of window piece w + 8 i: (window row, column);
        // window row r of kh group h is row r + h KHS of the full layout
        const uint32_t slot =
            (uint32_t)((w + NWV * i) * 1024 + 16 * lane) >> 5;
        const int rw_ = (int)fdiv(slot, g.fWp);
        const int cs = (int)slot - rw_ * g.Wp;
        const int r = rw_ + h * KHS;
        int j, lr;
        if (r < rc) {
          j = 0;
          lr = (int)oh0 + r;
        } else {
          const int qq = (int)fdiv((uint32_t)(r - rc), g.fHPd);
          j = 1 + qq;
          lr = r - rc - qq * g.HPd;
        }
        const int ih = lr - g.pt, iw = cs - g.pl;
        const uint32_t n = n0 + (uint32_t)j;
        const bool ok = w + NWV * i < NBP && rw_ < 1024 &&
                        cs < g.OW + KW - 1 && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W && n < (uint32_t)g.N;
        pwb[i] = ok ? (n * (uint32_t)g.H + (uint32_t)ih) * rowbytes +
                          (uint32_t)iw * pixbytes + gofs +
                          (uint32_t)(lane & 1) * 16u
                    : kBufOOB;
      }
    }
    d_h = h;
    d_cofs = (uint32_t)c * 32u;
    d_wofs = ((uint32_t)(gi * g.OCg + nt * BN) * (uint32_t)KT + c * 16) * 2u;
    d_bias = BIASB && bias && q == NQ - 1 && w == 0;
    d_bofs = lane < BN / 4 ? (uint32_t)(gi * g.OCg + nt * BN + 4 * lane) * 4u
                           : kBufOOB;
  };
  constexpr int NSLOT = NBW + NWW + (BIASB ? 1 : 0);
  const __amdgpu_buffer_rsrc_t rbias = dma_rsrc(bias);
  // this wave's window / weight pieces, opaque at each use (else one 64-bit
  // mask per slot is hoisted and spilled to VGPR lanes); an out-of-range
  // offset (kBufOOB = 2^31) plus a stage offset (< 2^31) stays past the
  // descriptor's records, so no select (conv_hc32 does the same)
  const int nb_live = (NBP - w + NWV - 1) / NWV;
  const int nw_live = (NWP - w + NWV - 1) / NWV;
  auto issue_slot = [&](int q, uint32_t stb) __attribute__((always_inline)) {
    // (the wide tiles keep the hoisted masks: opaque counts push their
    // 256-VGPR k-loop into more spills)
    constexpr bool OPQ = NJW <= 4;
    if (q < NBW) {
      int nb = nb_live;
      if constexpr (OPQ) asm volatile("" : "+s"(nb));
      if (q < nb)   // wave-uniform
        dma16(rs, smem + stb + (w + NWV * q) * 1024, pwb[q] + d_cofs);
    } else if (q < NBW + NWW) {
      if constexpr ((ABL & 256) != 0) {
        if (stb != 0 || d_cofs != 0) return;
      }
      const int i = q - NBW;
      int nw = nw_live;
      if constexpr (OPQ) asm volatile("" : "+s"(nw));
      if (i < nw) {   // wave-uniform
        const uint32_t o =
            (NH > 1 && d_h) ? wq(std::integral_constant<int, 1>{}, w + NWV * i)
                            : wq(std::integral_constant<int, 0>{}, w + NWV * i);
        dma16(rw, smem + stb + g.WIN + (w + NWV * i) * 1024, o + d_wofs);
      }
    } else if (d_bias) {
      // the item's bias block (natural channel order; lanes past BN / 4
      // read zeros)
      dma16(rbias, smem + stb + STAGE_B, d_bofs);
    }
  };
  // window slot bytes of this lane's pixels (fr of each m-tile)
  uint32_t bb[MI];
  auto slots = [&](int it) __attribute__((always_inline)) {
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
    const uint32_t n0 = fdiv(p0, g.fOHW);
    const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
    const int rc = g.OH - (int)oh0 + KH - 1;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const uint32_t p = p0 + wm * WPX + i * 16 + fr;
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
  const __amdgpu_buffer_rsrc_t ro = dma_rsrc(out);
  auto next = [&](int& it, int& q) __attribute__((always_inline)) {
    if (++q == NQ) {
      q = 0;
      it += nwg;
    }
  };
  prepare(item, 0);
#pragma unroll
  for (int q = 0; q < NSLOT; ++q) issue_slot(q, 0);
  slots(item);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // (it1, q1): the stage DMA'd into the other buffer during this one
  int it1 = item, q1 = 0;
  next(it1, q1);
  bool more1 = it1 < g.items;
  if (more1) prepare(it1, q1);

  f32x4 acc[MI][NJW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // The next stage's DMA slots are spread over the first ~2/3 of this
  // stage's k-steps (a burst at the stage start stalls both waves of a SIMD
  // at once: the barrier aligns them).  The bias and the derivative operand
  // of narrow tiles (NJW <= 3) are loaded into registers at the start of the
  // item's last stage; wide tiles read the bias from the stage's bias block
  // (DMA'd with the last stage) and the derivative operand from memory.
  constexpr bool PFA = NJW <= 3;
  float4 bpre[PFA ? NJW : 1];
  uint2 apre[PFA ? MI : 1][PFA ? NJW : 1];
  int q = 0;
  uint32_t cur = 0;
  // the k-steps of kh group H on the stage in buffer cur, interleaved with
  // the DMA of the next stage into nxt
  auto kloop = [&](auto hc, uint32_t nxt) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    constexpr int NKSH = H ? NKS1 : NKS0, TPH = H ? TP1 : TP0;
    // the k-steps the next stage's DMA is spread over: the first ~2/3
    // (ABL 16: the first third, 32: all of it at the first k-step)
    constexpr int NKSD = (ABL & 32)   ? 1
                         : (ABL & 16) ? (NKSH + 2) / 3
                         : NKSH > 2   ? (2 * NKSH + 2) / 3
                                      : NKSH;
    const uint32_t wb = cur + (uint32_t)g.WIN +
                        (uint32_t)(((wn * NJW) * 16 + fr) * (TPH * 32) +
                                   fq * 16);
    // narrow tiles: the fragments of k-step s + 1 are read before the MFMAs
    // of k-step s are issued (the compiler otherwise places every read next
    // to its MFMAs and waits out the LDS latency each k-step); wide tiles
    // have no registers for a second set
    constexpr bool SP = MI * NJW <= 24 && NH == 1 && (ABL & 64) == 0;
    auto rd = [&](int s, bf16x8* a, bf16x8* b) __attribute__((always_inline)) {
      const uint32_t os = H ? ofs1[H ? s : 0] : ofs0[s];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[i] = *(lds_bf16x8*)(sm + cur + bb[i] + os);
#pragma unroll
      for (int j = 0; j < NJW; ++j)
        b[j] = *(lds_bf16x8*)(sm + wb + j * 16 * (TPH * 32) + s * 64);
    };
    auto mfmas = [&](const bf16x8* a, const bf16x8* b)
                     __attribute__((always_inline)) {
      if constexpr ((ABL & 4) == 0) {
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
    };
    auto dma = [&](int s) __attribute__((always_inline)) {
      if constexpr ((ABL & 1) == 0) {
        if (more1) {
#pragma unroll
          for (int k = 0; k < NSLOT; ++k)
            if (k * NKSD / NSLOT == s) issue_slot(k, nxt);
        }
      }
    };
    if constexpr (SP) {
      bf16x8 a[2][MI], b[2][NJW];
      rd(0, a[0], b[0]);
#pragma unroll
      for (int s = 0; s < NKSH; ++s) {
        if (s + 1 < NKSH) rd(s + 1, a[(s + 1) & 1], b[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mfmas(a[s & 1], b[s & 1]);
        dma(s);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < NKSH; ++s) {
        bf16x8 a[MI], b[NJW];
        rd(s, a, b);
        mfmas(a, b);
        dma(s);
        // >= 24 accumulator tiles: no reads of the next k-step hoisted above
        // these MFMAs (double-buffered fragments would not fit the 256
        // registers of two waves per SIMD; the other wave hides the latency)
        if constexpr (MI * NJW >= 24 || NH > 1)
          __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (;;) {
    const bool last = q == NQ - 1;
    int ptl, gi, nt;
    decode(item, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
    // lane's first channel of store group u (within the n-tile): + 16 NG u
    const int chl = 16 * NG * wn * (NJW / NG) + 4 * NG * fq;
    const int chb = gi * g.OCg + nt * BN + chl;
    if constexpr (PFA) {
      if (last) {
        if (bias) {
#pragma unroll
          for (int j = 0; j < NJW; ++j)
            bpre[j] = *(const float4*)(bias + chb + 16 * NG * (j / NG) +
                                       4 * (j % NG));
        }
        if (aux) {
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const uint32_t p =
                min(p0 + wm * WPX + i * 16 + fr, (uint32_t)g.P - 1);
#pragma unroll
            for (int j = 0; j < NJW; ++j)
              apre[i][j] = *(const uint2*)(aux + (long long)p * g.OCT + chb +
                                           16 * NG * (j / NG) + 4 * (j % NG));
          }
        }
      }
    }
    // opaque per stage: otherwise the MI x NKS window addresses bb + ofs
    // are hoisted out of the stage loop into as many live registers
#pragma unroll
    for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(bb[i]));
    const uint32_t nxt = cur ^ STAGE;
    if (NH > 1 && (q % NH) != 0) kloop(std::integral_constant<int, 1>{}, nxt);
    else kloop(std::integral_constant<int, 0>{}, nxt);
    // stage (it1, q1) landed; every read of (item, q) done
    if constexpr ((ABL & 8) == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (last) {
      // lane: D[n = fq * 4 + r][m = fr] of each n-tile; with the row
      // permutation 4 NG consecutive output channels of one pixel per store
      // group: bias, activation, derivative of the layer below, bf16.
      // Buffer stores: pixels past the end go to the out-of-range offset
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const uint32_t p = p0 + wm * WPX + i * 16 + fr;
        const uint32_t pa = min(p, (uint32_t)g.P - 1);
        const bool ok = p < (uint32_t)g.P &&
                        !((ABL & 2) && acc[i][0][0] != 1234.5f);
        const uint32_t ob = (uint32_t)(((long long)p * g.OCT + chb) * 2);
#pragma unroll
        for (int u = 0; u < NJW / NG; ++u) {
          float v[4 * NG];
#pragma unroll
          for (int e = 0; e < NG; ++e) {
            float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (bias) {
              if constexpr (PFA) {
                bv = bpre[NG * u + e];
              } else {
                const f32x4 lb = *(const __attribute__((address_space(3)))
                                        f32x4*)(sm + cur + STAGE_B +
                                                (chl + 16 * NG * u + 4 * e) *
                                                    4);
                bv = make_float4(lb[0], lb[1], lb[2], lb[3]);
              }
            }
            v[4 * e] = acc[i][NG * u + e][0] + bv.x;
            v[4 * e + 1] = acc[i][NG * u + e][1] + bv.y;
            v[4 * e + 2] = acc[i][NG * u + e][2] + bv.z;
            v[4 * e + 3] = acc[i][NG * u + e][3] + bv.w;
          }
          act_fwd_n<4 * NG>(v, act);
          if (aux) {
            float y[4 * NG];
#pragma unroll
            for (int e = 0; e < NG; ++e) {
              uint2 av;
              if constexpr (PFA)
                av = apre[i][NG * u + e];
              else
                av = *(const uint2*)(aux + (long long)pa * g.OCT + chb +
                                     16 * NG * u + 4 * e);
              y[4 * e] = __uint_as_float(av.x << 16);
              y[4 * e + 1] = __uint_as_float(av.x & 0xffff0000u);
              y[4 * e + 2] = __uint_as_float(av.y << 16);
              y[4 * e + 3] = __uint_as_float(av.y & 0xffff0000u);
            }
            act_bwd_mul_n<4 * NG>(v, y, aux_act);
          }
          const uint32_t o = ob + 32 * NG * u;
          if constexpr (NG % 2 == 0) {   // 16-B aligned: 8 NG * 2 B apart
#pragma unroll
            for (int e = 0; e < NG; e += 2) {
              const uint4 qv = pack_bf16x8(v + 4 * e);
              __builtin_amdgcn_raw_buffer_store_b128(
                  u32x4{qv.x, qv.y, qv.z, qv.w}, ro,
                  ok ? o + 8 * e : kBufOOB, 0, 0);
            }
          } else {
#pragma unroll
            for (int e = 0; e < NG; ++e)
              __builtin_amdgcn_raw_buffer_store_b64(
                  u32x2{pack_bf16x2(v[4 * e], v[4 * e + 1]),
                        pack_bf16x2(v[4 * e + 2], v[4 * e + 3])},
                  ro, ok ? o + 8 * e : kBufOOB, 0, 0);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (more1) slots(it1);
    }
    if (!more1) break;
    item = it1;
    q = q1;
    next(it1, q1);
    more1 = it1 < g.items;
    if (more1) prepare(it1, q1);
    cur ^= STAGE;
  }
}

// ---------------------------------------------------------------------------
// conv_hc32: the same persistent window / chunk pipeline on the 32x32x16
// bf16 MFMA, where one K step is ONE tap x 16 channels (round 6, VERDICT r5
// "next" #1): a 3 x 3 stage is 9 MFMA k-steps instead of 5 two-tap 16x16x32
// steps of which one pads a zero-weight tap - 10 % of the MFMA issue and
// 2 of 11 weight granules per row (18 % of the stage's weight DMA) go away;
// a 5 x 5 stage loses 1 of 13 steps.  The 32x32 tile keeps the LDS-read /
// MFMA ratio of the 16x16 tiles (a 64 x 128 wave tile reads 2 window and 4
// weight fragments per 256 MFMA cycles).
//
// Lanes: B operand (pixels) lane l holds pixel l & 31 of the m-tile, k
// (channels) 8 (l >> 5) .. + 7 of the tap; A operand (weights) lane l holds
// LDS weight row l & 31 of the n-tile at the same k.  D[row][col] =
// D[oc][pixel]: lane l keeps rows (r & 3) + 8 (r >> 2) + 4 (l >> 5) of
// pixel l & 31; the weight rows are permuted so that these are the 16
// consecutive output channels 16 (l >> 5) + r of the n-tile (two 16-B
// stores per pixel and n-tile).
//
// Bank conflicts (ds_read_b128 lane groups {0-3,12-15,20-27}, ...): weight
// rows are T (odd) 32-B granules apart, so 8 consecutive rows sit on 8
// distinct even 16-B slots; the two 16-B halves of a granule are stored
// swapped on rows with bit 3 set, which puts rows r and r + 24 / r + 12
// and r + 20 of a lane group on distinct slots.  Window slots get the same
// half swap on slots with bit 3 set: 16 consecutive pixels then hit 16
// distinct bank slots (pixels that straddle a row wrap can still pair up).
// The DMA writes LDS linearly, so both swaps are applied to the SOURCE
// address and undone on the read (the same involution on both sides).
// ABL (diagnostic builds only, -DHVK_HC_ABL; tools/ablate_conv_hc.py): 1 no
// DMA after the first stage, 2 the next stage's DMA all at the first k-step,
// 4 no MFMAs, 8 no stage-end DMA wait, 16 the DMA spread over every k-step,
// 32 no epilogue stores, 64 no epilogue at all (1, 4, 8, 32, 64 give wrong
// results by design)
// MI: 32-pixel m-tiles per wave.  MI 2 with 8 waves (two per SIMD, 64 x
// NJ * 32 wave tiles).  MI 4 with 4 waves (one per SIMD, 128 x 128 wave
// tiles, accumulators in the AGPR half: a third less LDS read traffic per
// MFMA) compiles with 248 VGPRs spilled (hipcc, ROCm 7.2) and is not
// instantiated.
// Schedule variants measured and dropped (forced configurations, same
// process; profiles/r6/ab_hc32_schedule_variants_r6d.log,
// ab_hc32_branch_free_r6g.log): the SIMD partners (waves 4-7) walking each
// stage's taps rotated by T / 2 (0.1-0.9x: the doubled k-loop); s_setprio 1
// on them (+-2 %); a branch-free DMA issue with idle slots sent to a scratch
// piece (0.95-0.99x: the extra DMAs cost more than the branches).
template <int KH, int KW, int WM, int WN, int NJ, int NBW, int ABL = 0,
          int MI = 2, bool TS = false>
__global__ void __attribute__((
    amdgpu_flat_work_group_size(64 * WM * WN, 64 * WM * WN),
    amdgpu_waves_per_eu(WM * WN / 4, WM * WN / 4)))
conv_hc32_kernel(const uint16_t* __restrict__ src,
                 const uint16_t* __restrict__ wts,
                 const float* __restrict__ bias, uint16_t* __restrict__ out,
                 const uint16_t* __restrict__ aux, int act, int aux_act,
                 HcGeom g) {
  constexpr int T = KH * KW;
  static_assert(T % 2 == 1, "odd tap count: conflict-free weight rows");
  constexpr int NWV = WM * WN;
  static_assert(NWV == 8 || NWV == 4, "eight or four waves");
  constexpr int WPX = MI * 32;
  constexpr int TPX = WM * WPX;
  constexpr int BN = WN * NJ * 32;
  constexpr int RB = T * 32;                 // weight row bytes in LDS
  constexpr int WB = BN * RB;                // weight bytes per stage
  constexpr int NWP = (WB + 1023) / 1024;
  constexpr int NWW = (NWP + NWV - 1) / NWV;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  lds_u8* sm = (lds_u8*)smem;
  // stage: window | weights | bias block (1 KiB, the item's BN output
  // channels' bias, DMA'd with its last stage)
  const uint32_t STAGE_B = (uint32_t)g.WIN + NWP * 1024;
  const uint32_t STAGE = STAGE_B + 1024;
  const int NBP = g.WIN >> 10;
  const int NQ = g.CG >> 4;                  // K stages per item

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w % WM, wn = w / WM;
  const int l31 = lane & 31, lh = lane >> 5;

  // weight DMA: the stage's weights are one contiguous block of the packed
  // filter bank (hc32_pack_kernel: permuted rows, flipped taps and swapped
  // halves already in place), so a piece is a linear 1-KiB copy
  auto wq = [&](int pi) __attribute__((always_inline)) -> uint32_t {
    const uint32_t ib = (uint32_t)(pi * 1024 + 16 * lane);
    return ib < (uint32_t)WB ? ib : kBufOOB;
  };

  const __amdgpu_buffer_rsrc_t rs = dma_rsrc(src);
  const __amdgpu_buffer_rsrc_t rw = dma_rsrc(wts);
  const uint32_t rowbytes = (uint32_t)g.W * g.C * 2u;
  const uint32_t pixbytes = (uint32_t)g.C * 2u;

  auto decode = [&](int it, int& ptl, int& gi, int& nt)
                    __attribute__((always_inline)) {
    nt = it % g.NT;
    const int r = it / g.NT;
    gi = r % g.G;
    ptl = r / g.G;
  };
  uint32_t pwb[NBW];
  uint32_t d_cofs = 0, d_wofs = 0, d_bofs = 0;
  bool d_bias = false;
  auto prepare = [&](int it, int q) __attribute__((always_inline)) {
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    if (q == 0) {   // wave-uniform: a new item
      const uint32_t p0 = (uint32_t)ptl * TPX;
      const uint32_t n0 = fdiv(p0, g.fOHW);
      const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
      const int rc = g.OH - (int)oh0 + KH - 1;
      const uint32_t gofs = (uint32_t)(gi * g.CG) * 2u;
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        const uint32_t slot =
            (uint32_t)((w + NWV * i) * 1024 + 16 * lane) >> 5;
        const int r = (int)fdiv(slot, g.fWp);
        const int cs = (int)slot - r * g.Wp;
        int j, lr;
        if (r < rc) {
          j = 0;
          lr = (int)oh0 + r;
        } else {
          const int qq = (int)fdiv((uint32_t)(r - rc), g.fHPd);
          j = 1 + qq;
          lr = r - rc - qq * g.HPd;
        }
        const int ih = lr - g.pt, iw = cs - g.pl;
        const uint32_t n = n0 + (uint32_t)j;
        const bool ok = w + NWV * i < NBP && r < 1024 &&
                        cs < g.OW + KW - 1 && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W && n < (uint32_t)g.N;
        // stored half (lane & 1) swapped on slots with bit 3 set
        const uint32_t half = (uint32_t)((lane & 1) ^ ((slot >> 3) & 1));
        pwb[i] = ok ? (n * (uint32_t)g.H + (uint32_t)ih) * rowbytes +
                          (uint32_t)iw * pixbytes + gofs + half * 16u
                    : kBufOOB;
      }
    }
    d_cofs = (uint32_t)q * 32u;
    d_wofs = (uint32_t)(((gi * g.NT + nt) * NQ + q) * WB);
    d_bias = bias && q == NQ - 1 && w == 0;
    d_bofs = lane < BN / 4 ? (uint32_t)(gi * g.OCg + nt * BN + 4 * lane) * 4u
                           : kBufOOB;
  };
  constexpr int NSLOT = NBW + NWW + 1;
  const __amdgpu_buffer_rsrc_t rbias = dma_rsrc(bias);
  // this wave's window / weight pieces (one scalar each instead of a
  // wave-uniform mask per slot: those spilled to VGPR lanes)
  const int nb_live = (NBP - w + NWV - 1) / NWV;
  const int nw_live = (NWP - w + NWV - 1) / NWV;
  auto issue_slot = [&](int q, uint32_t stb, bool live)
                        __attribute__((always_inline)) {
    if (!live) return;
    // an out-of-range piece (kBufOOB = 2^31) plus a stage offset (< 2^31)
    // stays in [2^31, 2^32): still past the descriptor's records, no select
    // (opaque here: else the compiler hoists one 64-bit mask per slot)
    if (q < NBW) {
      int nb = nb_live;
      asm volatile("" : "+s"(nb));
      if (q < nb)   // wave-uniform
        dma16(rs, smem + stb + (w + NWV * q) * 1024, pwb[q] + d_cofs);
    } else if (q < NBW + NWW) {
      const int i = q - NBW;
      int nw = nw_live;
      asm volatile("" : "+s"(nw));
      if (i < nw)   // wave-uniform
        dma16(rw, smem + stb + g.WIN + (w + NWV * i) * 1024,
              wq(w + NWV * i) + d_wofs);
    } else if (d_bias) {
      dma16(rbias, smem + stb + STAGE_B, d_bofs);
    }
  };
  // window slot bytes of this lane's pixel in each m-tile
  uint32_t bb[MI];
  // the swizzled window byte offset of every (m-tile, tap) read, once per
  // item (MI * T VGPRs) instead of an add / shift / and / xor per read and
  // k-step (conv_hc32 loops +0-5 %, profiles/r6/ab_hc32_lean_loop_r6k.log)
  uint32_t ra[MI][T];
  const uint32_t wp32 = (uint32_t)g.Wp * 32u;
  auto slots = [&](int it) __attribute__((always_inline)) {
    int ptl, gi, nt;
    decode(it, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
    const uint32_t n0 = fdiv(p0, g.fOHW);
    const uint32_t oh0 = fdiv(p0 - n0 * (uint32_t)g.OHW, g.fOW);
    const int rc = g.OH - (int)oh0 + KH - 1;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const uint32_t p = p0 + wm * WPX + i * 32 + l31;
      if (p >= (uint32_t)g.P) {   // past the last pixel: slot 0 (finite)
        bb[i] = 16u * lh;
        continue;
      }
      const uint32_t n = fdiv(p, g.fOHW);
      const uint32_t pin = p - n * (uint32_t)g.OHW;
      const uint32_t oh = fdiv(pin, g.fOW);
      const int ow = (int)(pin - oh * (uint32_t)g.OW);
      const int j = (int)(n - n0);
      const int row = j == 0 ? (int)(oh - oh0) : rc + (j - 1) * g.HPd + (int)oh;
      bb[i] = (uint32_t)(row * g.Wp + ow) * 32u + 16u * lh;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int s = 0; s < T; ++s) {
        const uint32_t aa = bb[i] + (uint32_t)(s / KW) * wp32 +
                            (uint32_t)(s % KW) * 32u;
        ra[i][s] = aa ^ ((aa >> 4) & 16u);
      }
  };

  const int nwg = gridDim.x;
  int item = xcd_remap(blockIdx.x, nwg);
  if (item >= g.items) return;

  const __amdgpu_buffer_rsrc_t ro = dma_rsrc(out);
  auto next = [&](int& it, int& q) __attribute__((always_inline)) {
    if (++q == NQ) {
      q = 0;
      it += nwg;
    }
  };
  prepare(item, 0);
#pragma unroll
  for (int q = 0; q < NSLOT; ++q) issue_slot(q, 0, true);
  slots(item);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int it1 = item, q1 = 0;
  next(it1, q1);
  bool more1 = it1 < g.items;
  if (more1) prepare(it1, q1);

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const uint32_t wrow = (uint32_t)((wn * NJ * 32 + l31) * RB +
                                   16 * (lh ^ ((l31 >> 3) & 1)));
  int q = 0;
  uint32_t cur = 0;
  for (;;) {
    const bool last = q == NQ - 1;
    int ptl, gi, nt;
    decode(item, ptl, gi, nt);
    const uint32_t p0 = (uint32_t)ptl * TPX;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int s = 0; s < T; ++s) asm volatile("" : "+v"(ra[i][s]));
    const uint32_t nxt = cur ^ STAGE;
    const uint32_t wb = cur + (uint32_t)g.WIN + wrow;
    // the k-steps (taps) of this stage; the next stage's DMA slots spread
    // over the first ~2/3 of them
    constexpr int NKSD = (ABL & 2) ? 1 : (ABL & 16) ? T : (2 * T + 2) / 3;
    auto rd = [&](int s, bf16x8* a, bf16x8* b) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
        b[i] = *(lds_bf16x8*)(sm + cur + ra[i][s]);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        a[j] = *(lds_bf16x8*)(sm + wb + j * 32 * RB + s * 32);
    };
    // the stage's k-steps, taps in the order R, R + 1, ... (mod T)
    auto kloop = [&](auto rc) __attribute__((always_inline)) {
      constexpr int R = decltype(rc)::value;
      bf16x8 fa[2][NJ], fb[2][MI];
      rd(R % T, fa[0], fb[0]);
#pragma unroll
      for (int s = 0; s < T; ++s) {
        if (s + 1 < T)
          rd((s + 1 + R) % T, fa[(s + 1) & 1], fb[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((ABL & 4) == 0) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                  fa[s & 1][j], fb[s & 1][i], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            acc[i][0][0] += (float)fb[s & 1][i][0] + (float)fa[s & 1][0][0];
        }
        if constexpr ((ABL & 1) == 0) {
          if (more1) {
#pragma unroll
            for (int k = 0; k < NSLOT; ++k)
              if (k * NKSD / NSLOT == s) issue_slot(k, nxt, true);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    kloop(std::integral_constant<int, 0>{});
    // stage (it1, q1) landed; every read of (item, q) done
    if constexpr ((ABL & 8) == 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (last) {
      // lane: pixel l31 of each m-tile, output channels 16 lh + r of each
      // n-tile (the row permutation): bias, activation, derivative of the
      // layer below, two 16-B bf16 stores; pixels past the end go to the
      // out-of-range offset
      const int chl = wn * NJ * 32 + 16 * lh;   // within the item's BN
      const int chb = gi * g.OCg + nt * BN + chl;
      if constexpr ((ABL & 64) != 0) {   // keeps the MFMAs live
        float z = 0.f;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) z += acc[i][j][0];
        if (z == 1234.5f) out[t] = 0;
      }
      // EM 1: strict ReLU forward without a derivative operand, 2: linear
      // with the strict-ReLU derivative (the AlexNet backward-data), both on
      // the packed bf16 (relu_bf16x2 / relu_mask_bf16x2); 0: any
      // activation in f32.  The epilogue stalls every MFMA of the CU
      // (ablation: 8-9 % of the forward, 28 % of conv5 backward-data).
      // LDS staging slot of this wave in the consumed stage buffer (free
      // until the barrier below): 32 rows of NJ * 64 B + 16 B pad (the pad
      // spreads the rows' 16-B pieces over the banks)
      constexpr int TSR = NJ * 64 + 16;
      const uint32_t tsb = cur + (uint32_t)(w * 32 * TSR);
      auto epi = [&](auto emc) __attribute__((always_inline)) {
        constexpr int EM = decltype(emc)::value;
        // every derivative operand of the epilogue loaded before its first
        // store: the compiler cannot move a global load above a buffer store
        // (possible alias), so per-block loads serialised the epilogue on a
        // load and a store round trip per block (vmcnt counts both, in
        // order).  The k-loop's fragment registers are dead here.
        // (the 128-channel tile keeps per-block loads: hoisted, even per
        // m-tile, they spill its 251-VGPR k-loop)
        constexpr bool HALL = MI * NJ <= 6;
        constexpr int AI = (EM == 1 || !HALL) ? 1 : MI;
        constexpr int AJ = (EM == 1 || !HALL) ? 1 : NJ;
        uint4 avs[AI][AJ][2];
        auto ld_aux = [&](int i, int j, uint4& a0, uint4& a1)
                          __attribute__((always_inline)) {
          const uint32_t pa =
              min(p0 + wm * WPX + i * 32 + l31, (uint32_t)g.P - 1);
          const uint16_t* ap = aux + (long long)pa * g.OCT + chb + 32 * j;
          a0 = *(const uint4*)ap;
          a1 = *(const uint4*)(ap + 8);
        };
        if (EM != 1 && HALL && aux) {
#pragma unroll
          for (int i = 0; i < ((ABL & 64) || EM == 1 ? 0 : MI); ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              ld_aux(i, j, avs[i % AI][j % AJ][0], avs[i % AI][j % AJ][1]);
        }
        auto get_aux = [&](int i, int j, uint4& a0, uint4& a1)
                           __attribute__((always_inline)) {
          if constexpr (HALL) {
            a0 = avs[i % AI][j % AJ][0];
            a1 = avs[i % AI][j % AJ][1];
          } else {
            ld_aux(i, j, a0, a1);
          }
        };
        // one call per m-tile (a lambda on a constant: the loop form was
        // too large for the unroller once the staged stores were added,
        // and a rolled loop puts the accumulators in scratch)
        auto epi_i = [&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          const uint32_t p = p0 + wm * WPX + i * 32 + l31;
          const bool ok = p < (uint32_t)g.P;
          const uint32_t ob = (uint32_t)(((long long)p * g.OCT + chb) * 2);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float v[16];
#pragma unroll
            for (int e = 0; e < 16 && EM == 2; ++e) v[e] = acc[i][j][e];
#pragma unroll
            for (int e = 0; e < 16 && EM != 2; e += 4) {
              float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
              if (bias) {
                const f32x4 lb = *(const __attribute__((address_space(3)))
                                        f32x4*)(sm + cur + STAGE_B +
                                                (chl + 32 * j + e) * 4);
                bv = make_float4(lb[0], lb[1], lb[2], lb[3]);
              }
              v[e] = acc[i][j][e] + bv.x;
              v[e + 1] = acc[i][j][e + 1] + bv.y;
              v[e + 2] = acc[i][j][e + 2] + bv.z;
              v[e + 3] = acc[i][j][e + 3] + bv.w;
            }
            uint32_t pk[8];
            if constexpr (EM == 0) {
              act_fwd_n<16>(v, act);
              if (aux) {
                float y[16];
                uint4 a0, a1;
                get_aux(i, j, a0, a1);
                const uint32_t av[8] = {a0.x, a0.y, a0.z, a0.w,
                                        a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                  y[2 * e] = __uint_as_float(av[e] << 16);
                  y[2 * e + 1] = __uint_as_float(av[e] & 0xffff0000u);
                }
                act_bwd_mul_n<16>(v, y, aux_act);
              }
#pragma unroll
              for (int e = 0; e < 8; ++e)
                pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]);
            } else if constexpr (EM == 1) {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                pk[e] = relu_bf16x2(pack_bf16x2(v[2 * e], v[2 * e + 1]));
            } else {
              uint4 a0, a1;
              get_aux(i, j, a0, a1);
              const uint32_t av[8] = {a0.x, a0.y, a0.z, a0.w,
                                      a1.x, a1.y, a1.z, a1.w};
#pragma unroll
              for (int e = 0; e < 8; ++e)
                pk[e] = pack_bf16x2(v[2 * e], v[2 * e + 1]) &
                        relu_mask_bf16x2(av[e]);
            }
            if constexpr (TS) {   // stage the m-tile in LDS
#pragma unroll
              for (int e = 0; e < 2; ++e)
                *(lds_u32x4*)(sm + tsb + l31 * TSR + (32 * j + 16 * lh + 8 * e) *
                                                         2) =
                    u32x4{pk[4 * e], pk[4 * e + 1], pk[4 * e + 2],
                          pk[4 * e + 3]};
            } else {
              const uint32_t o = ob + 64 * j;
#pragma unroll
              for (int e = 0; e < 2; ++e)
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{pk[4 * e], pk[4 * e + 1], pk[4 * e + 2],
                          pk[4 * e + 3]},
                    ro,
                    ok && !((ABL & 32) && v[0] != 1234.5f) ? o + 16 * e
                                                            : kBufOOB,
                    0, 0);
            }
          }
          if constexpr (TS) {
            // the wave's 32 pixels x NJ * 32 channels read back as rows of
            // 16-B chunks: lanes on consecutive chunks of a pixel's run, so
            // a store covers runs of NJ * 64 contiguous bytes instead of 64
            // scattered 16-B pieces (its own LDS slot: no barrier)
            // (lane opaque here: else the chunk addresses, lane constants,
            // are hoisted out of the item loop and spill its k-loop)
            int ln = lane;
            asm volatile("" : "+v"(ln));
#pragma unroll
            for (int k = 0; k < 2 * NJ; ++k) {
              const int c = ln + 64 * k;   // chunk of the m-tile
              const int row = c / (4 * NJ), col = c - row * (4 * NJ);
              const u32x4 val = *(const lds_u32x4*)(sm + tsb + row * TSR +
                                                     col * 16);
              const uint32_t pr = p0 + wm * WPX + i * 32 + row;
              const uint32_t go =
                  (uint32_t)(((long long)pr * g.OCT + chb - 16 * lh) * 2) +
                  col * 16;
              __builtin_amdgcn_raw_buffer_store_b128(
                  val, ro,
                  pr < (uint32_t)g.P && !((ABL & 32) && val[0] == 12345u)
                      ? go : kBufOOB,
                  0, 0);
            }
          }
        };
        if constexpr ((ABL & 64) == 0) {
          static_assert(MI <= 4, "m-tiles of the epilogue");
          epi_i(std::integral_constant<int, 0>{});
          if constexpr (MI > 1) epi_i(std::integral_constant<int, 1>{});
          if constexpr (MI > 2) epi_i(std::integral_constant<int, 2>{});
          if constexpr (MI > 3) epi_i(std::integral_constant<int, 3>{});
        }
      };
      if (!aux && act == ACT_STRICT_RELU)
        epi(std::integral_constant<int, 1>{});
      else if (aux && act == ACT_LINEAR && aux_act == ACT_STRICT_RELU && !bias)
        epi(std::integral_constant<int, 2>{});
      else
        epi(std::integral_constant<int, 0>{});
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
      if (more1) slots(it1);
      // the staging slots lie in the buffer the next stage's DMA fills
      if constexpr (TS) __builtin_amdgcn_s_barrier();
    }
    if (!more1) break;
    item = it1;
    q = q1;
    next(it1, q1);
    more1 = it1 < g.items;
    if (more1) prepare(it1, q1);
    cur ^= STAGE;
  }
}

// Stage-major filter bank of conv_hc32: packed[g][nt][c][n][t][16] holds,
// for n-tile nt of group g and 16-channel chunk c, LDS weight row n (output
// channel g OCg + nt BN + perm(n), the epilogue's row permutation), tap t
// (flipped for backward-data) and source channels 16 c .. + 15, with the two
// 8-channel halves swapped on rows with bit 3 set - exactly the stage's LDS
// image, so the kernel's weight DMA is a contiguous copy.  The per-(row,
// tap) 32-B gather it replaces touched one 128-B line per 32 B in L2.
// src: [OCT][T][CG] (the forward filter bank, or backward-data's permutation
// wt[g][c][kh][kw][oc], which has the same shape for the transposed conv).
// fwd_w (backward-data only): src is the forward filter bank [G][CG][T][OCg]
// itself, not its [G][OCg][T][CG] permutation; the pack gathers each piece's
// 8 reduction channels at their stride (the permute pass is not needed)
__global__ void hc32_pack_kernel(const uint16_t* __restrict__ src,
                                 uint16_t* __restrict__ dst, int T, int CG,
                                 int OCg, int BN, int flip,
                                 long long pieces, int fwd_w) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= pieces) return;
  const int hs = (int)(q & 1);
  long long r = q >> 1;
  const int tp = (int)(r % T);
  r /= T;
  const int n = (int)(r % BN);
  r /= BN;
  const int NQ = CG >> 4;
  const int c = (int)(r % NQ);
  r /= NQ;
  const int NT = OCg / BN;
  const int nt = (int)(r % NT);
  const int gi = (int)(r / NT);
  const int rr = n & 31;
  const int o = gi * OCg + nt * BN + (n & ~31) + 16 * ((rr >> 2) & 1) +
                4 * (rr >> 3) + (rr & 3);
  const int half = hs ^ ((n >> 3) & 1);
  const int tap = flip ? T - 1 - tp : tp;
  uint4 v;
  if (fwd_w) {
    const uint16_t* wp = src + ((long long)(gi * CG + c * 16 + half * 8) * T +
                                tap) * OCg + (o - gi * OCg);
    const long long st = (long long)T * OCg;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)wp[2 * j * st] | ((uint32_t)wp[(2 * j + 1) * st] << 16);
    v = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    v = *(const uint4*)(src + ((long long)o * T + tap) * CG + c * 16 +
                        half * 8);
  }
  *(uint4*)(dst + q * 8) = v;
}

struct HcPlan {
  int var;      // 0: not taken
  size_t lds;
  int grid;
  HcGeom g;
  int KH, KW;
  void* wpack;  // conv_hc32: the stage-major filter bank workspace
  int fwd_w;    // backward-data weights in the forward layout (hc32_pack)
};

constexpr int kCUs = 256;
constexpr int kNBW = 8;   // window pieces per wave: 64 KiB windows at most
// -2 automatic on the shapes where it beats the implicit-GEMM kernels, -1 on
// every shape it supports, 0 off, > 0 one forced configuration
int g_hc_variant = -2;
int g_hc_abl = 0;         // diagnostic instantiation (configurations 5-7)
// window slot row pitch Wp = OW + pad (hvk_hc_pitch_pad; pad >= KW - 1).  8
// keeps Wp = OW (mod 8): conflict-free A fragments across row wraps; a
// smaller pad shrinks the window of small images (13 x 13: 21 -> 15 slots
// per row) at the price of conflicts on the wrapping fragments
int g_hc_pad = 8;

// m32: conv_hc32_kernel (32x32x16 MFMA, NJW = 32-channel n-tiles per
// wave), else conv_hc_kernel (16x16x32, NJW = 16-channel n-tiles)
struct HcCand { int var, KH, KW, KHS, WM, WN, NJW, NBW, m32, mi = 2; };
// conv_hc32 candidates on (hvk_hc32; default on), else only conv_hc_kernel
int g_hc32 = 1;
int g_hc_last = 0;   // configuration of the last conv_hc launch (tests)
int g_hc32_ts = 1;   // conv_hc32 epilogue stores staged through LDS
// per kernel size, in order of preference (the first whose n-tile divides
// the group's outputs and whose two stages fit the LDS)
constexpr HcCand kHcCands[] = {
    // conv_hc32: one tap x 16 channels per MFMA k-step
    {21, 3, 3, 3, 8, 1, 4, 5, 1},   // 512 px x 128 ch
    {22, 3, 3, 3, 8, 1, 3, 5, 1},   // 512 px x 96 ch
    {23, 3, 3, 3, 8, 1, 2, 8, 1},   // 512 px x 64 ch
    // 5 x 5 (AlexNet conv2 forward), 512 px x 64 ch: 25 k-steps per stage,
    // no pad tap; fits the LDS only with the tight window pitch (below)
    {24, 5, 5, 5, 8, 1, 2, 4, 1},

    {6, 3, 3, 3, 8, 1, 8, 5, 0},   // 512 px x 128 ch: AlexNet conv3 / 5 fwd, conv3 dgrad
    {7, 3, 3, 3, 8, 1, 6, 5, 0},   // 512 px x 96 ch: conv1 (s2d), conv4 fwd, conv4 / 5 dgrad
    {1, 3, 3, 3, 4, 2, 4, 8, 0},   // 256 px x 128 ch
    {2, 3, 3, 3, 4, 2, 3, 8, 0},   // 256 px x 96 ch
    {3, 3, 3, 3, 8, 1, 4, 8, 0},   // 512 px x 64 ch: VGG-16 64-channel layers
    {11, 5, 5, 5, 8, 1, 2, 8, 0},  // 512 px x 32 ch: AlexNet conv2 fwd
    {4, 5, 5, 5, 4, 2, 2, 8, 0},   // 256 px x 64 ch
    {5, 5, 5, 5, 8, 1, 3, 8, 0},   // 512 px x 48 ch: AlexNet conv2 dgrad
    // 512 px x 64 ch in two kh groups (3 + 2 rows per stage): half the
    // weights per stage, but twice the window DMA and stages; AlexNet conv2
    // forward 755 TF against 878 for configuration 4 (forced runs only)
    {8, 5, 5, 3, 8, 1, 4, 8, 0},
};

int hc_bn(const HcCand& k) { return k.WN * k.NJW * (k.m32 ? 32 : 16); }

// weight (+ bias block) bytes of one stage
int hc_nbytes_w(const HcCand& k) {
  const int T = k.KHS * k.KW;
  if (k.m32) return (hc_bn(k) * T * 32 + 1023) / 1024 * 1024 + 1024;
  const int TP = 2 * ((T + 1) / 2) + 1;
  const int BN = k.WN * k.NJW * 16;
  return (BN * TP * 32 + 1023) / 1024 * 1024 + (k.NJW <= 3 ? 0 : 1024);
}

HcPlan hc_plan(int N, int H, int W, int C, int OH, int OW, int OCT, int KH,
               int KW, int pt, int pl, int groups, bool flip, bool al16) {
  HcPlan p{};
  HcGeom& g = p.g;
  if (g_hc_variant == 0) return p;
  const int CG = C / groups, OCg = OCT / groups;
  if (CG % 16 || OCg % 16 || OCT % 4) return p;
  // automatic: every shape except the ones measured slower than the T4 /
  // 256x256 / 128-row implicit GEMM in one process
  // (profiles/r5/ab_conv_hc_alexnet_vgg_r5o.log): AlexNet conv1 1.16x,
  // conv2 1.12x / 1.45x (forward / backward-data), conv3-5 1.02-1.05x, VGG
  // conv1_2 forward 1.08x, conv3_2 1.06-1.07x, conv4_2 1.00-1.02x; left to
  // the GEMM: VGG conv1_2 backward-data (0.99x) and conv2_2 (0.95x)
  if (g_hc_variant == -2 && ((flip && CG <= 64) || (OW >= 100 && CG >= 128)))
    return p;
  if ((long long)N * H * W * C * 2 >= kBufMaxBytes) return p;
  if ((long long)N * OH * OW * OCT * 2 >= kBufMaxBytes) return p;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.OCT = OCT;
  g.OCg = OCg; g.CG = CG; g.pt = pt; g.pl = pl; g.G = groups;
  g.P = N * OH * OW;
  g.OHW = OH * OW;
  g.Wp = OW + std::max(g_hc_pad, KW - 1);
  g.HPd = OH + KH - 1;
  g.flip = flip ? 1 : 0;
  if (OW + KW - 1 > g.Wp || g.Wp >= (1 << 20)) return p;
  for (const HcCand& k : kHcCands) {
    if (k.KH != KH || k.KW != KW) continue;
    // the 5 x 5 conv_hc32 tile: Wp = OW + 4 (OW + 8 overflows the LDS by
    // 6 KiB at 27 x 27; the row-wrap fragments then share some banks)
    g.Wp = OW + ((k.m32 && k.KW == 5) ? KW - 1 : std::max(g_hc_pad, KW - 1));
    if (g_hc_variant > 0 && k.var != g_hc_variant) continue;
    // conv_hc32: 16-B stores / derivative loads, and at least three K
    // stages per item (its bias block lives in the stage buffers: with
    // fewer, a fast wave's bias DMA for the next item could overwrite the
    // block a slow wave still reads in its epilogue)
    if (k.m32 && (!g_hc32 || !al16 || CG < 48 || OCT % 8)) continue;
    if (!k.m32 && k.NJW > 3 && CG < 48) continue;
    const int BN = hc_bn(k), TPX = k.WM * (k.m32 ? 32 * k.mi : 64);
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
      wr = std::max(wr, row + k.KHS);   // the first kh group's rows
    }
    if (wr >= 1024) continue;
    g.WIN = (wr * g.Wp * 32 + 1023) / 1024 * 1024;
    if (g.WIN / 1024 > k.WM * k.WN * k.NBW) continue;
    const size_t lds = 2 * (size_t)(g.WIN + hc_nbytes_w(k));
    if (lds > 160 * 1024) continue;
    // conv_hc32's store staging: one 32-row slot per wave in the window and
    // weight part of a stage buffer; backward-data only (same process,
    // profiles/r6/ab_hc32_staged_stores_r6y.log: conv3 / conv5 dgrad +3.4 /
    // +2.8 %, the forwards -4 % (conv1) to +0.8 %)
    g.ts = k.m32 && flip && g_hc32_ts &&
           k.WM * k.WN * 32 * (k.NJW * 64 + 16) <=
               g.WIN + hc_nbytes_w(k) - 1024;
    g.NT = OCg / BN;
    g.items = (int)(tiles * groups * g.NT);
    g.fOW = make_fastdiv(OW);
    g.fOHW = make_fastdiv(g.OHW);
    g.fHPd = make_fastdiv(g.HPd);
    g.fWp = make_fastdiv(g.Wp);
    p.lds = lds;
    p.grid = std::min(g.items, kCUs);
    p.var = k.var;
    p.KH = KH;
    p.KW = KW;
    return p;
  }
  return p;
}

template <int KH, int KW, int KHS, int WM, int WN, int NJW, int ABL = 0,
          int NBW = kNBW>
hipError_t go_hc(const HcPlan& p, const void* src, const void* wts,
                 const float* bias, void* out, const void* aux, int act,
                 int aux_act, hipStream_t s) {
  if (p.g.WIN / 1024 > WM * WN * NBW) return hipErrorInvalidValue;
  auto kern = conv_hc_kernel<KH, KW, KHS, WM, WN, NJW, NBW, ABL>;
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

// packed filter-bank bytes of a conv_hc32 plan (0: not a conv_hc32 plan)
long long hc32_wpack_bytes(const HcPlan& p) {
  if (p.var < 21) return 0;
  const int KH = p.KH, KW = p.KW;
  return (long long)p.g.G * p.g.OCg * KH * KW * p.g.CG * 2;
}

template <int KH, int KW, int WM, int WN, int NJ, int NBW, int ABL = 0,
          int MI = 2, bool TS = false>
hipError_t go_hc32_ts(const HcPlan& p, const void* src, const void* wts,
                   const float* bias, void* out, const void* aux, int act,
                   int aux_act, hipStream_t s) {
  if (p.g.WIN / 1024 > WM * WN * NBW) return hipErrorInvalidValue;
  if (p.wpack == nullptr) return hipErrorInvalidValue;
  {   // the stage-major filter bank, stream-ordered before the conv
    const long long pieces = hc32_wpack_bytes(p) / 16;
    hipLaunchKernelGGL(hc32_pack_kernel, dim3((unsigned)((pieces + 255) / 256)),
                       dim3(256), 0, s, (const uint16_t*)wts,
                       (uint16_t*)p.wpack, KH * KW, p.g.CG, p.g.OCg,
                       WN * NJ * 32, p.g.flip, pieces, p.fwd_w);
    wts = p.wpack;
  }
  auto kern = conv_hc32_kernel<KH, KW, WM, WN, NJ, NBW, ABL, MI, TS>;
  static bool attr = false;   // once per instantiation, before any capture
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(
        (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
        160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)p.grid), dim3(64 * WM * WN), p.lds, s,
                     (const uint16_t*)src, (const uint16_t*)wts, bias,
                     (uint16_t*)out, (const uint16_t*)aux, act, aux_act, p.g);
  return launch_status(s);
}

template <int KH, int KW, int WM, int WN, int NJ, int NBW, int ABL = 0>
hipError_t go_hc32(const HcPlan& p, const void* src, const void* wts,
                   const float* bias, void* out, const void* aux, int act,
                   int aux_act, hipStream_t s) {
  if (p.g.ts)
    return go_hc32_ts<KH, KW, WM, WN, NJ, NBW, ABL, 2, true>(
        p, src, wts, bias, out, aux, act, aux_act, s);
  return go_hc32_ts<KH, KW, WM, WN, NJ, NBW, ABL, 2, false>(
      p, src, wts, bias, out, aux, act, aux_act, s);
}

#ifdef HVK_HC_ABL
template <int KH, int KW, int WM, int WN, int NJ, int NBW>
hipError_t go_hc32_abl(const HcPlan& p, const void* src, const void* wts,
                       const float* bias, void* out, const void* aux, int act,
                       int aux_act, hipStream_t s) {
  switch (g_hc_abl) {
#define HC32_ABL(A) \
    case A: return go_hc32<KH, KW, WM, WN, NJ, NBW, A>(                       \
        p, src, wts, bias, out, aux, act, aux_act, s);
    HC32_ABL(1) HC32_ABL(2) HC32_ABL(4) HC32_ABL(8) HC32_ABL(16) HC32_ABL(32)
    HC32_ABL(9) HC32_ABL(64)
#undef HC32_ABL
    default: return go_hc32<KH, KW, WM, WN, NJ, NBW, 0>(
        p, src, wts, bias, out, aux, act, aux_act, s);
  }
}
#endif

// a production launch with an explicit NBW (go_hc's seventh parameter is
// the ablation selector)
template <int KH, int KW, int KHS, int WM, int WN, int NJW, int NBW = kNBW>
hipError_t go_hc_nbw(const HcPlan& p, const void* src, const void* wts,
                     const float* bias, void* out, const void* aux, int act,
                     int aux_act, hipStream_t s) {
  return go_hc<KH, KW, KHS, WM, WN, NJW, 0, NBW>(p, src, wts, bias, out, aux,
                                                  act, aux_act, s);
}

#ifdef HVK_HC_ABL
template <int KH, int KW, int KHS, int WM, int WN, int NJW, int NBW = kNBW>
hipError_t go_hc_abl(const HcPlan& p, const void* src, const void* wts,
                     const float* bias, void* out, const void* aux, int act,
                     int aux_act, hipStream_t s) {
  switch (g_hc_abl) {
#define HC_ABL(A) \
    case A: return go_hc<KH, KW, KHS, WM, WN, NJW, A, NBW>(                    \
        p, src, wts, bias, out, aux, act, aux_act, s);
    HC_ABL(1) HC_ABL(2) HC_ABL(4) HC_ABL(8) HC_ABL(3) HC_ABL(9) HC_ABL(16)
    HC_ABL(32) HC_ABL(64) HC_ABL(256)
#undef HC_ABL
    default: return go_hc<KH, KW, KHS, WM, WN, NJW, 0, NBW>(
        p, src, wts, bias, out, aux, act, aux_act, s);
  }
}

#endif  // HVK_HC_ABL

hipError_t hc_launch(const HcPlan& p, const void* src, const void* wts,
                     const float* bias, void* out, const void* aux, int act,
                     int aux_act, hipStream_t s) {
  switch (p.var) {
#define HC_GO(V, ...) \
    case V: return go_hc<__VA_ARGS__>(p, src, wts, bias, out, aux, act, \
                                      aux_act, s);
#ifdef HVK_HC_ABL
#define HC_GO_ABL(V, ...) \
    case V: return go_hc_abl<__VA_ARGS__>(p, src, wts, bias, out, aux, act, \
                                          aux_act, s);
#define HC32(V, ...) \
    case V: return go_hc32_abl<__VA_ARGS__>(p, src, wts, bias, out, aux, \
                                            act, aux_act, s);
#else
#define HC_GO_ABL(V, ...) \
    case V: return go_hc_nbw<__VA_ARGS__>(p, src, wts, bias, out, aux, act, \
                                          aux_act, s);
#define HC32(V, ...) \
    case V: return go_hc32<__VA_ARGS__>(p, src, wts, bias, out, aux, act, \
                                        aux_act, s);
#endif
    HC_GO(1, 3, 3, 3, 4, 2, 4)
    HC_GO(2, 3, 3, 3, 4, 2, 3)
    HC_GO(3, 3, 3, 3, 8, 1, 4)
    HC_GO(4, 5, 5, 5, 4, 2, 2)
    HC_GO_ABL(5, 5, 5, 5, 8, 1, 3)
    HC_GO_ABL(6, 3, 3, 3, 8, 1, 8, 5)
    HC_GO_ABL(7, 3, 3, 3, 8, 1, 6, 5)
    HC_GO(8, 5, 5, 3, 8, 1, 4)
    HC_GO_ABL(11, 5, 5, 5, 8, 1, 2)
    HC32(21, 3, 3, 8, 1, 4, 5)
    HC32(22, 3, 3, 8, 1, 3, 5)
    HC32(23, 3, 3, 8, 1, 2, 8)
    HC32(24, 5, 5, 8, 1, 2, 4)

#undef HC32
#undef HC_GO_ABL
#undef HC_GO
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// -2 automatic (the measured winners), -1 every supported shape, 0 off,
// > 0 one forced configuration (kHcCands var).
HVK_API void hvk_hc_variant(int v) { g_hc_variant = v; }
// Diagnostic ablation builds of configurations 5, 6 and 7 (see conv_hc_kernel's
// ABL); 0 = the production kernel.
HVK_API void hvk_hc_ablation(int a) { g_hc_abl = a; }
// window row pitch pad (8 default; see g_hc_pad)
HVK_API void hvk_hc_pitch_pad(int p) { g_hc_pad = p; }
// conv_hc32 candidates (32x32x16 MFMA, one tap per k-step): 1 on (default),
// 0 only the 16x16x32 kernel
HVK_API void hvk_hc32(int on) { g_hc32 = on; }
// conv_hc32 epilogue stores: 1 staged through LDS (default), 0 direct
HVK_API void hvk_hc32_ts(int on) { g_hc32_ts = on; }
// configuration (kHcCands var) of the last hvk_conv_{fwd,dgrad}_hc launch
HVK_API int hvk_hc_last_variant() { return g_hc_last; }

// Forward: Y[N][OH][OW][OC] = act(conv(X, W) + bias), stride 1, X bf16 NHWC,
// W [OC][KH][KW][C/g].  Returns 0, -2 when the shape does not take this
// kernel (the caller falls back), or a HIP error.
namespace {
HcPlan hc_plan_fwd(int N, int H, int W, int C, int OC, int KH, int KW, int pt,
                   int pl, int OH, int OW, int groups, bool al16) {
  return hc_plan(N, H, W, C, OH, OW, OC, KH, KW, pt, pl, groups, false, al16);
}
// the window source is dY (OH x OW, OC channels), the output dX (H x W, C
// channels), origin KH - 1 - pt / KW - 1 - pl
HcPlan hc_plan_dgrad(int N, int H, int W, int C, int OC, int KH, int KW,
                     int pt, int pl, int OH, int OW, int groups, bool al16) {
  return hc_plan(N, OH, OW, OC, H, W, C, KH, KW, KH - 1 - pt, KW - 1 - pl,
                 groups, true, al16);
}
}  // namespace

// Bytes of the conv_hc32 packed filter-bank workspace the call with this
// geometry needs (0: it does not take conv_hc32).  dgrad: the backward-data
// geometry (hvk_conv_dgrad_hc's arguments); aligned: the output (and the
// derivative operand) are 16-B aligned.
HVK_API long long hvk_conv_hc_wpack_bytes(int dgrad, int N, int H, int W,
                                          int C, int OC, int KH, int KW,
                                          int pt, int pl, int OH, int OW,
                                          int groups, int aligned) {
  HcPlan p = dgrad ? hc_plan_dgrad(N, H, W, C, OC, KH, KW, pt, pl, OH, OW,
                                   groups, aligned != 0)
                   : hc_plan_fwd(N, H, W, C, OC, KH, KW, pt, pl, OH, OW,
                                 groups, aligned != 0);
  return p.var ? hc32_wpack_bytes(p) : 0;
}

// wpack: the packed filter-bank workspace (hvk_conv_hc_wpack_bytes; may be
// null when that is 0)
HVK_API int hvk_conv_fwd_hc(const void* X, const void* Wt, const float* bias,
                            void* Y, int N, int H, int W, int C, int OC,
                            int KH, int KW, int pt, int pl, int OH, int OW,
                            int groups, int act, void* wpack, hipStream_t s) {
  if (((uintptr_t)X & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)Y & 7) ||
      ((uintptr_t)bias & 15) || ((uintptr_t)wpack & 15))
    return -2;
  HcPlan p = hc_plan_fwd(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
                         ((uintptr_t)Y & 15) == 0);
  if (!p.var || (hc32_wpack_bytes(p) && !wpack)) return -2;
  p.wpack = wpack;
  g_hc_last = p.var;
  return (int)hc_launch(p, X, Wt, bias, Y, nullptr, act, 0, s);
}

// Backward-data: dX[N][H][W][C] = conv^T(dY, W) [* act'(aux)], stride 1,
// from the dgrad weight permutation wt[g][c][kh][kw][oc].  -2: not taken.
HVK_API int hvk_conv_dgrad_hc(const void* dY, const void* Wt, void* dX, int N,
                              int H, int W, int C, int OC, int KH, int KW,
                              int pt, int pl, int OH, int OW, int groups,
                              const void* aux, int aux_act, void* wpack,
                              hipStream_t s) {
  if (((uintptr_t)dY & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)dX & 7) ||
      ((uintptr_t)aux & 7) || ((uintptr_t)wpack & 15))
    return -2;
  HcPlan p = hc_plan_dgrad(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
                           ((uintptr_t)dX & 15) == 0 &&
                               ((uintptr_t)aux & 15) == 0);
  if (!p.var || (hc32_wpack_bytes(p) && !wpack)) return -2;
  p.wpack = wpack;
  p.fwd_w = 0;
  g_hc_last = p.var;
  return (int)hc_launch(p, dY, Wt, nullptr, dX, aux, 0, aux_act, s);
}

// hvk_conv_dgrad_hc with the weights in the FORWARD layout W [OC][KH][KW][Cg]:
// the conv_hc32 plans pack them straight into their filter bank; -3 when the
// plan is not a conv_hc32 one (the caller permutes and uses hvk_conv_dgrad_hc)
HVK_API int hvk_conv_dgrad_hc_w(const void* dY, const void* W_, void* dX,
                                int N, int H, int W, int C, int OC, int KH,
                                int KW, int pt, int pl, int OH, int OW,
                                int groups, const void* aux, int aux_act,
                                void* wpack, hipStream_t s) {
  if (((uintptr_t)dY & 15) || ((uintptr_t)dX & 7) || ((uintptr_t)aux & 7) ||
      ((uintptr_t)wpack & 15))
    return -2;
  HcPlan p = hc_plan_dgrad(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
                           ((uintptr_t)dX & 15) == 0 &&
                               ((uintptr_t)aux & 15) == 0);
  if (!p.var) return -2;
  if (!hc32_wpack_bytes(p)) return -3;
  if (!wpack) return -2;
  p.wpack = wpack;
  p.fwd_w = 1;
  g_hc_last = p.var;
  return (int)hc_launch(p, dY, W_, nullptr, dX, aux, 0, aux_act, s);
}
