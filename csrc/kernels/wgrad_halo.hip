// wgrad_halo.hip - convolution weight gradient with the input window of a
// pixel step staged ONCE in LDS and shared by every tap ("halo" wgrad).
//
//   dW[oc][kh][kw][c] (+)= sum_p dY[p][oc] * X[n(p)][oh(p)+kh-pt][ow(p)+kw-pl][c]
//
// Why (round 5, VERDICT r4 "next" #1): the GEMM formulation of the weight
// gradient (gemm_core.h ConvWgradB, T4) stages im2col(X) = KH*KW shifted
// copies of the same pixels through LDS-DMA every K step.  The DMA pieces,
// not the MFMAs, bound those loops (profiles/r4/t4_ablation/README.md:
// without the main-loop DMA +62-73 % on the weight gradients).  Here a
// workgroup owns an output tile of MT output channels x (KHT*KW taps x NP
// 16-channel planes) and loops over a range of pixels in steps of 64; per
// step it DMAs
//   * A = dY[64 pixels][MT channels]  (MN-major, 64 x MT bf16), and
//   * the input WINDOW those 64 pixels touch: the image rows they span plus
//     the kh halo, all columns plus the kw halo, NP x 16 channels -
// and every tap reads its B fragments out of the same window at a constant
// offset (kh * Wp + kw slots).  Per step that is ~30 KiB for 64 x MT x
// (KHT*KW*16*NP) MACs: 3x3, MT 128, NP 2 -> 0.0058 operand bytes per FLOP
// against 0.013 for the T4 loop and 0.0156 for the 128-row loop.
//
// Window layout (per plane, 32-B slots of 16 bf16 channels): slot
// rs * Wp + cs holds input pixel (row of window row rs, column cs - pl).
// With Wp = OW + 8 (congruent to OW mod 8) 8 consecutive output pixels -
// across an output-row wrap too - map to 8 slots that are distinct mod 8:
// the ds_read_b64_tr_b16 lane groups (8 pixels x 32 B) hit every bank once.
// The default is the tight Wp = OW + KW - 1 (g_halo_pad): conflicts only on
// the lane groups that straddle a row wrap, and fewer window bytes.
// Window row rs of a step starting at output row oh0 of image n0 is input
// row oh0 + kh0 - pt + rs of image n0 while rs < OH - oh0 + KHT - 1, and
// input row rs - (OH - oh0) - (KHT - 1) + kh0 - pt of image n0 + 1 after
// that (the second image's rows shifted by the halo so the images never
// share a slot).  A step spans at most two images (OH * OW >= 64), and one
// when OH * OW is a multiple of 64 (the window then has no second image).
//
// K order.  MFMA 16x16x32 k labels map to pixels pi(l) = (l & 4 ? 16 : 0) +
// (l >> 3) * 4 + (l & 3) (+32 per half step) on BOTH operands, so each
// 32-lane group of a transposed read covers 8 consecutive pixels (the
// conflict-free shape above).  The sum over pixels is order-independent
// up to f32 rounding: results match the 128-row loop to rounding, not bits.
//
// Split over pixels: each workgroup stores its f32 tile into its own slice
// of a [splits][OC][KK] workspace (no atomics), and hvk_wgrad_finish adds
// the slices in split order into dW - deterministic.  The bias gradient
// comes from extra MFMAs against an all-ones operand in the workgroups of
// tap group 0 / channel chunk 0 (slices [splits][OC]).
//
// Reference counterpart: the GD units' err x input matmuls through OCLBLAS
// (/root/reference/veles/ocl_blas.py:187-236); SURVEY §2.4 row 1.
#include "conv_geom.h"

// diagnostic builds only (wrong results by design): 1 no window DMA, 2 no
// epilogue stores, 4 no MFMAs
#ifndef HVK_HALO_ABL
#define HVK_HALO_ABL 0
#endif
#include "fp8_common.h"

using namespace hvk;

namespace {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct HaloGeom {
  int N, H, W, C, OH, OW, OC, Cg, OCg, KH, KW, pt, pl;
  int P;     // N * OH * OW
  int OHW;   // OH * OW
  int KK;    // KH * KW * Cg
  int Wp;    // pixel-slot row pitch (OW + 8)
  int WR;    // full-row window: rows
  int SEGP;  // segment window: slots per kh segment
  int spi;   // segment window: 64-pixel steps per image
  FastDiv fOW, fWp;
};

// XOR of the 32-B block index of A image row r (MT / 16 blocks per row):
// 8 consecutive rows (one 32-lane transposed read) hit every bank once
template <int MT>
__device__ __forceinline__ int a_sw(int r) {
  if constexpr (MT == 128) return r & 7;
  else if constexpr (MT == 96) return (r >> 2) & 1;
  else return (r >> 1) & 3;   // 64, 192
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;

// two transposed 8-B reads (k rows of this lane's pixel, +16 pixels) ->
// one 16x16x32 operand fragment; o0 / o1 are LDS byte offsets
__device__ __forceinline__ bf16x8 tr_read(lds_u8* sm, uint32_t o0,
                                          uint32_t o1) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sm + o0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(sm + o1));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// MT: output channels per tile; NP: 16-channel planes; KHT: kh rows per tap
// group; KW: taps per kh row; NJW: n-tiles (16 columns) per wave column;
// PB: LDS bytes per window plane.
// SEG: the segment window for wide images (64 pixels cover a sliver of two
// rows): steps are image-aligned (a step never crosses an image; the last
// one of an image is partial) and each kh has its own SEGP-slot segment,
// slot kh * SEGP + d + kw for the pixel at slot distance d = (oh - oh0) *
// Wp + ow - ow0 from the step's first pixel - the same "pixel base + tap
// offset" read with the tap row pitch SEGP instead of Wp.  kspan counts
// steps then, pixels otherwise.
template <int MT, int NP, int KHT, int KW, int NJW, int PB, bool SEG>
__global__ void __launch_bounds__(256, 2)
wgrad_halo_kernel(const uint16_t* __restrict__ x,
                  const uint16_t* __restrict__ dy, float* __restrict__ ws,
                  float* __restrict__ wsb, HaloGeom g, int mtiles,
                  int cchunks, int kgroups, int tiles, int kspan,
                  int bias) {
  constexpr int NJ = KHT * KW * NP;          // n-tiles of the workgroup
  static_assert(2 * NJW >= NJ, "two wave columns cover the n-tiles");
  constexpr int MI = MT / 32;                // m-tiles per wave (2 x 2 waves)
  constexpr int AP = MT * 2;                 // A image row pitch (bytes)
  constexpr int ABYTES = 64 * AP;
  constexpr int NA = ABYTES / 1024;          // A DMA pieces per step
  static_assert(NA % 4 == 0, "A pieces divide over the four waves");
  constexpr int NAW = NA / 4;
  constexpr int BBYTES = NP * PB;
  constexpr int NB = (BBYTES + 1023) / 1024; // window DMA pieces per step
  constexpr int NBW = (NB + 3) / 4;
  constexpr int STAGE = ABYTES + NB * 1024;
  static_assert(2 * 2 * STAGE <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int split = wgid / tiles;
  int tt = tile;
  const int kg = tt % kgroups; tt /= kgroups;
  const int cc = tt % cchunks; tt /= cchunks;
  const int mt = tt % mtiles;
  const int gi = tt / mtiles;
  // pixel range (full-row window) or step range (segment window)
  const int total = SEG ? g.N * g.spi : g.P;
  const int pbeg = split * kspan;
  const int pend = min(total, pbeg + kspan);
  if (pbeg >= pend) return;   // the host sizes splits so this never happens
  const int coff_y = gi * g.OCg + mt * MT;
  const int coff_x = gi * g.Cg + cc * 16 * NP;
  const int kh0 = kg * KHT;

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int trq = fr >> 2, trp = fr & 3;
  const int q = fq * 4 + trq;   // this lane's pixel (+16 h + 32 ks)

  lds_u8* sm = (lds_u8*)smem;
  const __amdgpu_buffer_rsrc_t ra = dma_rsrc(dy);
  const __amdgpu_buffer_rsrc_t rb = dma_rsrc(x);

  // ---- A DMA slots: image byte -> (row r, logical 8-channel chunk)
  uint32_t a_off[NAW];
  int a_row[NAW];
#pragma unroll
  for (int i = 0; i < NAW; ++i) {
    const int ib = (w * NAW + i) * 1024 + 16 * lane;
    const int r = ib / AP;
    const int pc = (ib - r * AP) >> 4;
    const int lb = (pc >> 1) ^ a_sw<MT>(r);
    const int m = lb * 16 + (pc & 1) * 8;
    a_row[i] = r;
    a_off[i] = (uint32_t)(r * g.OC + coff_y + m) * 2u;
  }
  // ---- window DMA slots: image byte -> (plane, window row, column, half)
  // (full-row) or (plane, kh segment, segment slot, half) (SEG)
  const int WS = SEG ? KHT * g.SEGP : g.WR * g.Wp;
  int b_rs[NBW];
  uint32_t b_col[NBW];
  uint32_t b_ok[NBW];
  int b_j[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int pi = w + 4 * i;
    const int ib = pi * 1024 + 16 * lane;
    const int plane = ib / PB;
    const int wb = ib - plane * PB;
    const int slot = wb >> 5;
    const int half = (wb >> 4) & 1;
    if constexpr (SEG) {
      const int khs = slot / g.SEGP;
      b_rs[i] = khs;   // the segment's kh
      b_j[i] = slot - khs * g.SEGP;
      b_ok[i] = (pi < NB && plane < NP && slot < WS) ? 1u : 0u;
      b_col[i] = (uint32_t)(coff_x + plane * 16 + half * 8) * 2u;
    } else {
      const int rs = slot / g.Wp;
      const int cs = slot - rs * g.Wp;
      const int iw = cs - g.pl;
      b_rs[i] = rs;
      b_j[i] = 0;
      b_ok[i] = (pi < NB && plane < NP && slot < WS &&
                 cs < g.OW + g.KW - 1 && iw >= 0 && iw < g.W) ? 1u : 0u;
      b_col[i] = (uint32_t)(iw * g.C + coff_x + plane * 16 + half * 8) * 2u;
    }
  }
  const uint32_t rowbytes = (uint32_t)g.W * g.C * 2u;
  const uint32_t pixbytes = (uint32_t)g.C * 2u;

  // ---- A fragment offsets (bytes in the A image) of this lane's m-tiles
  const int mrow0 = wr * (MT / 2);
  int a_frag[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mb = mrow0 / 16 + i;
    a_frag[i] = q * AP + ((mb ^ a_sw<MT>(q)) << 5) + trp * 8;
  }

  f32x4 acc[MI][NJW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                       (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};

  // step decode (wave-uniform): the first pixel's image n, its index pin
  // in the image, row and column
  uint32_t n0, pin0, oh0, ow0;
  if constexpr (SEG) {
    n0 = (uint32_t)pbeg / (uint32_t)g.spi;
    pin0 = ((uint32_t)pbeg - n0 * g.spi) * 64u;
  } else {
    n0 = (uint32_t)pbeg / (uint32_t)g.OHW;
    pin0 = (uint32_t)pbeg - n0 * g.OHW;
  }
  oh0 = fdiv(pin0, g.fOW);
  ow0 = pin0 - oh0 * g.OW;

  // DMA of the step at (n, pin, oh, ow) into stage st
  auto issue = [&](int n, int pin, int oh, int ow, uint8_t* st) {
    if constexpr ((HVK_HALO_ABL & 1) != 0) return;
    const int p = n * g.OHW + pin;
    const uint32_t pa = (uint32_t)p * (uint32_t)g.OC * 2u;
    const int plim = SEG ? g.OHW - pin : pend - p;   // valid rows < plim
#pragma unroll
    for (int i = 0; i < NAW; ++i) {
      const uint32_t v = (a_row[i] < plim) ? pa + a_off[i] : kBufOOB;
      dma16(ra, st + (w * NAW + i) * 1024, v);
    }
    if constexpr (SEG) {
      // segment kh, slot j: input row oh + (ow + j) / Wp + kh0 + kh - pt,
      // column (ow + j) % Wp - pl
      const int ihb = oh + kh0 - g.pt;
      const uint32_t nrow = (uint32_t)n * g.H;
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        if (w + 4 * i < NB) {   // wave-uniform
          const uint32_t sj = (uint32_t)(ow + b_j[i]);
          const uint32_t rr = fdiv(sj, g.fWp);
          const int col = (int)(sj - rr * (uint32_t)g.Wp);
          const int ih = ihb + (int)rr + b_rs[i];
          const int iw = col - g.pl;
          const bool ok = b_ok[i] && col < g.OW + g.KW - 1 &&
                          (unsigned)iw < (unsigned)g.W &&
                          (unsigned)ih < (unsigned)g.H;
          const uint32_t v = ok ? (nrow + (uint32_t)ih) * rowbytes +
                                      (uint32_t)iw * pixbytes + b_col[i]
                                : kBufOOB;
          dma16(rb, st + ABYTES + (w + 4 * i) * 1024, v);
        }
      }
      return;
    }
    // window rows: image n up to row slot rc, image n + 1 after it
    const int rc = g.OH - oh + KHT - 1;
    const int ih_a = oh + kh0 - g.pt;
    const int ih_b = kh0 - g.pt - rc;
    const int gr_a = n * g.H + ih_a;
    const int gr_b = (n + 1) * g.H + ih_b;
    const bool n1ok = n + 1 < g.N;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (w + 4 * i < NB) {   // wave-uniform
        const int rs = b_rs[i];
        const bool first = rs < rc;
        const int ih = (first ? ih_a : ih_b) + rs;
        const int gr = (first ? gr_a : gr_b) + rs;
        const bool ok = b_ok[i] && (unsigned)ih < (unsigned)g.H &&
                        (first || n1ok);
        const uint32_t v = ok ? (uint32_t)gr * rowbytes + b_col[i] : kBufOOB;
        dma16(rb, st + ABYTES + (w + 4 * i) * 1024, v);
      }
    }
  };
  auto advance = [&](uint32_t& n, uint32_t& pin, uint32_t& oh,
                     uint32_t& ow) {
    pin += 64;
    if (SEG && pin >= (uint32_t)g.OHW) {   // the next image's first step
      pin = 0; oh = 0; ow = 0; ++n;
      return;
    }
    if (!SEG && pin >= (uint32_t)g.OHW) pin -= g.OHW;
    ow += 64;
    while (ow >= (uint32_t)g.OW) {   // scalar: at most 64 / OW + 1 turns
      ow -= g.OW;
      if (++oh == (uint32_t)g.OH) { oh = 0; ++n; }
    }
  };

  const int nk = SEG ? pend - pbeg : (pend - pbeg + 63) >> 6;
  issue(n0, pin0, oh0, ow0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  uint32_t nn = n0, pinn = pin0, ohn = oh0, own = ow0;
  advance(nn, pinn, ohn, own);

  const bool bwave = bias && kg == 0 && cc == 0 && wc == 0;

  auto main_loop = [&](auto wcc, auto with_bias) {
    constexpr int WC = decltype(wcc)::value;
    constexpr bool WB = decltype(with_bias)::value;
    for (int kt = 0; kt < nk; ++kt) {
      const uint32_t cur = (kt & 1) * STAGE;
      if (kt + 1 < nk)
        issue(nn, pinn, ohn, own, smem + ((kt + 1) & 1) * STAGE);
      // B fragment bases (LDS bytes) of this lane's 4 pixels (q + 16 i)
      // for every kh of the tap group
      uint32_t bb[4][KHT];
      const int kp = SEG ? g.SEGP : g.Wp;   // slots per kh
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t ow = ow0 + q + 16 * i;
        const uint32_t gr = fdiv(ow, g.fOW);
        const int owr = (int)(ow - gr * (uint32_t)g.OW);
        int slot;
        if constexpr (SEG) {
          // pixels past the image end (A rows zero) read slot 0 of the
          // stage: finite data, never the other stage's unwritten LDS
          slot = pin0 + q + 16 * i < (uint32_t)g.OHW
                     ? (int)gr * g.Wp + owr - (int)ow0 : 0;
        } else {
          slot = ((int)gr + ((oh0 + gr >= (uint32_t)g.OH) ? KHT - 1 : 0)) *
                     g.Wp + owr;
        }
        const uint32_t base = cur + ABYTES + slot * 32 + trp * 8;
#pragma unroll
        for (int kh = 0; kh < KHT; ++kh) bb[i][kh] = base + kh * kp * 32;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const uint32_t oa = cur + a_frag[i] + ks * 32 * AP;
          a[i] = tr_read(sm, oa, oa + 16 * AP);
        }
#pragma unroll
        for (int j = 0; j < NJW; ++j) {
          const int jg = WC * NJW + j;
          if (jg < NJ) {   // compile-time after unrolling (WC constant)
            const int tl = jg / NP, pl_ = jg - (jg / NP) * NP;
            const int khl = tl / KW, kwl = tl - (tl / KW) * KW;
            const uint32_t off = kwl * 32 + pl_ * PB;   // bytes
            const bf16x8 b = tr_read(sm, bb[2 * ks][khl] + off,
                                     bb[2 * ks + 1][khl] + off);
            if constexpr ((HVK_HALO_ABL & 4) != 0) {
              acc[0][j][0] += (float)b[0] + (float)a[0][0];
            } else {
#pragma unroll
              for (int i = 0; i < MI; ++i)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    b, a[i], acc[i][j], 0, 0, 0);
            }
          }
        }
        if constexpr (WB) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, a[i],
                                                              accb[i], 0, 0, 0);
        }
      }
      // step kt + 1 landed; every read of step kt done
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      ow0 = own; oh0 = ohn; n0 = nn; pin0 = pinn;
      advance(nn, pinn, ohn, own);
    }
  };
  if (wc == 0) {
    if (bwave) main_loop(std::integral_constant<int, 0>{}, std::true_type{});
    else main_loop(std::integral_constant<int, 0>{}, std::false_type{});
  } else {
    main_loop(std::integral_constant<int, 1>{}, std::false_type{});
  }

  // ---- epilogue: D[n][m] quads (4 consecutive n of one m) -> slice
  const long long sbase = (long long)split * g.OC;
#pragma unroll
  for (int j = 0; j < NJW; ++j) {
    const int jg = wc * NJW + j;
    if (jg >= NJ || ((HVK_HALO_ABL & 2) && acc[0][j][0] != 1234.5f)) continue;
    const int tl = jg / NP, pl_ = jg - (jg / NP) * NP;
    const int khg = kh0 + tl / KW, kwl = tl - (tl / KW) * KW;
    const int ng = (khg * g.KW + kwl) * g.Cg + cc * 16 * NP + pl_ * 16 + fq * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int mg = coff_y + mrow0 + i * 16 + fr;
      *(float4*)(ws + (sbase + mg) * g.KK + ng) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if (bwave && fq == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
      wsb[sbase + coff_y + mrow0 + i * 16 + fr] = accb[i][0];
  }
}

// dW[e] += sum_s ws[s][e] (e < n4 float4 elements), dbias[m] += sum_s
// wsb[s][m]: R threads per element sum the splits k = r, r + R, ... and
// their partials are added in r order (deterministic).  R > 1 when the
// splits outnumber the elements' parallelism (AlexNet conv1: one tile, 512
// splits: one thread per element took 0.24 ms).  Blocks past nmain reduce
// the bias.
template <int R>
__global__ void __launch_bounds__(256)
wgrad_finish_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                    long long n4, int splits, const float* __restrict__ wsb,
                    float* __restrict__ db, int oc, int nmain) {
  constexpr int EPB = 256 / R;
  __shared__ float4 red[256];
  const int r = threadIdx.x % R, el = threadIdx.x / R;
  if ((int)blockIdx.x < nmain) {
    const long long e = (long long)blockIdx.x * EPB + el;
    float4 sacc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < n4)
      for (int k = r; k < splits; k += R) {
        const float4 v = ((const float4*)ws)[(long long)k * n4 + e];
        sacc.x += v.x; sacc.y += v.y; sacc.z += v.z; sacc.w += v.w;
      }
    if constexpr (R == 1) {
      if (e < n4) {
        float4 d = ((float4*)dw)[e];
        d.x += sacc.x; d.y += sacc.y; d.z += sacc.z; d.w += sacc.w;
        ((float4*)dw)[e] = d;
      }
      return;
    }
    red[threadIdx.x] = sacc;
    __syncthreads();
    if (r == 0 && e < n4) {
      float4 t = red[el * R];
#pragma unroll
      for (int i = 1; i < R; ++i) {
        const float4 v = red[el * R + i];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      float4 d = ((float4*)dw)[e];
      d.x += t.x; d.y += t.y; d.z += t.z; d.w += t.w;
      ((float4*)dw)[e] = d;
    }
    return;
  }
  if (db == nullptr) return;
  const int m = ((int)blockIdx.x - nmain) * EPB + el;
  float sb = 0.f;
  if (m < oc)
    for (int k = r; k < splits; k += R) sb += wsb[(long long)k * oc + m];
  float* rf = (float*)red;
  rf[threadIdx.x] = sb;
  __syncthreads();
  if (r == 0 && m < oc) {
    float t = rf[el * R];
    for (int i = 1; i < R; ++i) t += rf[el * R + i];
    db[m] += t;
  }
}

// ---------------------------------------------------------------------------
// fp8 (f8f6f4) form: dW += sum_p dY8[p][oc] X8[...][c] / (s_dY s_X) on
// v_mfma_scale_f32_16x16x128_f8f6f4 (twice the bf16 rate), from the e5m2 /
// e4m3 copies the fp8 forward and backward-data already hold (the operands
// of wgrad_fp8.hip).  Same window scheme with 1-byte elements: steps of 128
// pixels, 16-B window slots of 16 channels, Wp = OW + 16 (congruent to OW
// mod 16: 16 consecutive pixels -> 16 slots distinct mod 16, so each
// half-wave of a ds_read_b64_tr_b8 - 16 pixels x 16 B - hits every bank
// once).  The 32 k labels 32 g + 8 j + q of lane group g (read j, row q)
// map to pixel 64 (g >> 1) + 16 j + 8 (g & 1) + q on both operands, which
// makes those 16 pixels consecutive.  A image: [128 pixels][MT oc] with the
// 16-B chunk c of row r at c ^ f8(r).
template <int MT>
__device__ __forceinline__ int a_sw8(int r) {
  if constexpr (MT == 128) return (r >> 1) & 7;
  else return (r >> 2) & 3;   // 64
}

typedef __attribute__((ext_vector_type(8))) int i32x8h;
typedef __attribute__((ext_vector_type(2))) int i32x2h;
typedef __attribute__((address_space(3))) i32x2h lds_i32x2;

__device__ __forceinline__ i32x2h tr8(lds_u8* sm, uint32_t o) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)(sm + o));
}

template <int MT, int NP, int KHT, int KW, int NJW, int PB, bool SEG, int FX,
          int FDY>
__global__ void __launch_bounds__(256, 2)
wgrad_halo8_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ dy,
                   float* __restrict__ ws, float* __restrict__ wsb,
                   HaloGeom g, int mtiles, int cchunks, int kgroups, int tiles,
                   int kspan, int bias, const float* sxs, const float* sdys,
                   int hist, float fmax_x, float fmax_dy) {
  constexpr int STEP = 128;
  constexpr int NJ = KHT * KW * NP;
  static_assert(2 * NJW >= NJ, "two wave columns cover the n-tiles");
  constexpr int MI = MT / 32;
  constexpr int AP = MT;                     // A row pitch (bytes)
  constexpr int ABYTES = STEP * AP;
  constexpr int NA = ABYTES / 1024;
  static_assert(NA % 4 == 0, "A pieces divide over the four waves");
  constexpr int NAW = NA / 4;
  constexpr int NB = (NP * PB + 1023) / 1024;
  constexpr int NBW = (NB + 3) / 4;
  constexpr int STAGE = ABYTES + NB * 1024;
  static_assert(2 * 2 * STAGE <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int split = wgid / tiles;
  int tt = tile;
  const int kg = tt % kgroups; tt /= kgroups;
  const int cc = tt % cchunks; tt /= cchunks;
  const int mt = tt % mtiles;
  const int gi = tt / mtiles;
  const int total = SEG ? g.N * g.spi : g.P;
  const int pbeg = split * kspan;
  const int pend = min(total, pbeg + kspan);
  if (pbeg >= pend) return;
  const int coff_y = gi * g.OCg + mt * MT;
  const int coff_x = gi * g.Cg + cc * 16 * NP;
  const int kh0 = kg * KHT;

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int qq = fr >> 1, pp = fr & 1;
  // pixel of read j: pix0 + 16 j
  const int pix0 = 64 * (fg >> 1) + 8 * (fg & 1) + qq;

  lds_u8* sm = (lds_u8*)smem;
  const __amdgpu_buffer_rsrc_t ra = dma_rsrc(dy);
  const __amdgpu_buffer_rsrc_t rb = dma_rsrc(x);

  uint32_t a_off[NAW];
  int a_row[NAW];
#pragma unroll
  for (int i = 0; i < NAW; ++i) {
    const int ib = (w * NAW + i) * 1024 + 16 * lane;
    const int r = ib / AP;
    const int pc = (ib - r * AP) >> 4;
    const int lc = pc ^ a_sw8<MT>(r);
    a_row[i] = r;
    a_off[i] = (uint32_t)(r * g.OC + coff_y + lc * 16);
  }
  const int WS = SEG ? KHT * g.SEGP : g.WR * g.Wp;
  int b_rs[NBW];
  uint32_t b_col[NBW];
  uint32_t b_ok[NBW];
  int b_j[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int pi = w + 4 * i;
    const int ib = pi * 1024 + 16 * lane;
    const int plane = ib / PB;
    const int wb = ib - plane * PB;
    const int slot = wb >> 4;
    if constexpr (SEG) {
      const int khs = slot / g.SEGP;
      b_rs[i] = khs;
      b_j[i] = slot - khs * g.SEGP;
      b_ok[i] = (pi < NB && plane < NP && slot < WS) ? 1u : 0u;
      b_col[i] = (uint32_t)(coff_x + plane * 16);
    } else {
      const int rs = slot / g.Wp;
      const int cs = slot - rs * g.Wp;
      const int iw = cs - g.pl;
      b_rs[i] = rs;
      b_j[i] = 0;
      b_ok[i] = (pi < NB && plane < NP && slot < WS &&
                 cs < g.OW + g.KW - 1 && iw >= 0 && iw < g.W) ? 1u : 0u;
      b_col[i] = (uint32_t)(iw * g.C + coff_x + plane * 16);
    }
  }
  const uint32_t rowbytes = (uint32_t)g.W * g.C;
  const uint32_t pixbytes = (uint32_t)g.C;

  const int mrow0 = wr * (MT / 2);
  int a_frag[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int mb = mrow0 / 16 + i;
    a_frag[i] = pix0 * AP + ((mb ^ a_sw8<MT>(pix0)) << 4) + 8 * pp;
  }

  f32x4 acc[MI][NJW];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int one8 = FX == 0 ? 0x38383838 : 0x3C3C3C3C;   // 1.0 in X's format
  const i32x8h ones = {one8, one8, one8, one8, one8, one8, one8, one8};

  uint32_t n0, pin0, oh0, ow0;
  if constexpr (SEG) {
    n0 = (uint32_t)pbeg / (uint32_t)g.spi;
    pin0 = ((uint32_t)pbeg - n0 * g.spi) * STEP;
  } else {
    n0 = (uint32_t)pbeg / (uint32_t)g.OHW;
    pin0 = (uint32_t)pbeg - n0 * g.OHW;
  }
  oh0 = fdiv(pin0, g.fOW);
  ow0 = pin0 - oh0 * g.OW;

  auto issue = [&](int n, int pin, int oh, int ow, uint8_t* st) {
    const int p = n * g.OHW + pin;
    const uint32_t pa = (uint32_t)p * (uint32_t)g.OC;
    const int plim = SEG ? g.OHW - pin : pend - p;
#pragma unroll
    for (int i = 0; i < NAW; ++i) {
      const uint32_t v = (a_row[i] < plim) ? pa + a_off[i] : kBufOOB;
      dma16(ra, st + (w * NAW + i) * 1024, v);
    }
    if constexpr (SEG) {
      const int ihb = oh + kh0 - g.pt;
      const uint32_t nrow = (uint32_t)n * g.H;
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        if (w + 4 * i < NB) {
          const uint32_t sj = (uint32_t)(ow + b_j[i]);
          const uint32_t rr = fdiv(sj, g.fWp);
          const int col = (int)(sj - rr * (uint32_t)g.Wp);
          const int ih = ihb + (int)rr + b_rs[i];
          const int iw = col - g.pl;
          const bool ok = b_ok[i] && col < g.OW + g.KW - 1 &&
                          (unsigned)iw < (unsigned)g.W &&
                          (unsigned)ih < (unsigned)g.H;
          const uint32_t v = ok ? (nrow + (uint32_t)ih) * rowbytes +
                                      (uint32_t)iw * pixbytes + b_col[i]
                                : kBufOOB;
          dma16(rb, st + ABYTES + (w + 4 * i) * 1024, v);
        }
      }
      return;
    }
    const int rc = g.OH - oh + KHT - 1;
    const int ih_a = oh + kh0 - g.pt;
    const int ih_b = kh0 - g.pt - rc;
    const int gr_a = n * g.H + ih_a;
    const int gr_b = (n + 1) * g.H + ih_b;
    const bool n1ok = n + 1 < g.N;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (w + 4 * i < NB) {
        const int rs = b_rs[i];
        const bool first = rs < rc;
        const int ih = (first ? ih_a : ih_b) + rs;
        const int grow = (first ? gr_a : gr_b) + rs;
        const bool ok = b_ok[i] && (unsigned)ih < (unsigned)g.H &&
                        (first || n1ok);
        const uint32_t v = ok ? (uint32_t)grow * rowbytes + b_col[i] : kBufOOB;
        dma16(rb, st + ABYTES + (w + 4 * i) * 1024, v);
      }
    }
  };
  auto advance = [&](uint32_t& n, uint32_t& pin, uint32_t& oh,
                     uint32_t& ow) {
    pin += STEP;
    if (SEG && pin >= (uint32_t)g.OHW) {
      pin = 0; oh = 0; ow = 0; ++n;
      return;
    }
    if (!SEG && pin >= (uint32_t)g.OHW) pin -= g.OHW;
    ow += STEP;
    while (ow >= (uint32_t)g.OW) {
      ow -= g.OW;
      if (++oh == (uint32_t)g.OH) { oh = 0; ++n; }
    }
  };

  const int nk = SEG ? pend - pbeg : (pend - pbeg + STEP - 1) / STEP;
  issue(n0, pin0, oh0, ow0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  uint32_t nn = n0, pinn = pin0, ohn = oh0, own = ow0;
  advance(nn, pinn, ohn, own);
  const bool bwave = bias && kg == 0 && cc == 0 && wc == 0;

  auto main_loop = [&](auto wcc, auto with_bias) {
    constexpr int WC = decltype(wcc)::value;
    constexpr bool WB = decltype(with_bias)::value;
    for (int kt = 0; kt < nk; ++kt) {
      const uint32_t cur = (kt & 1) * STAGE;
      if (kt + 1 < nk)
        issue(nn, pinn, ohn, own, smem + ((kt + 1) & 1) * STAGE);
      const int kp = SEG ? g.SEGP : g.Wp;
      uint32_t bb[4][KHT];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t ow = ow0 + pix0 + 16 * j;
        const uint32_t gr = fdiv(ow, g.fOW);
        const int owr = (int)(ow - gr * (uint32_t)g.OW);
        int slot;
        if constexpr (SEG) {
          slot = pin0 + pix0 + 16 * j < (uint32_t)g.OHW
                     ? (int)gr * g.Wp + owr - (int)ow0 : 0;
        } else {
          slot = ((int)gr + ((oh0 + gr >= (uint32_t)g.OH) ? KHT - 1 : 0)) *
                     g.Wp + owr;
        }
        const uint32_t base = cur + ABYTES + slot * 16 + 8 * pp;
#pragma unroll
        for (int kh = 0; kh < KHT; ++kh) bb[j][kh] = base + kh * kp * 16;
      }
      i32x8h a[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const i32x2h h = tr8(sm, cur + a_frag[i] + 16 * j * AP);
          a[i][2 * j] = h[0];
          a[i][2 * j + 1] = h[1];
        }
      }
#pragma unroll
      for (int jn = 0; jn < NJW; ++jn) {
        const int jg = WC * NJW + jn;
        if (jg < NJ) {
          const int tl = jg / NP, pl_ = jg - (jg / NP) * NP;
          const int khl = tl / KW, kwl = tl - (tl / KW) * KW;
          const uint32_t off = kwl * 16 + pl_ * PB;
          i32x8h b;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const i32x2h h = tr8(sm, bb[j][khl] + off);
            b[2 * j] = h[0];
            b[2 * j + 1] = h[1];
          }
#pragma unroll
          for (int i = 0; i < MI; ++i)
            acc[i][jn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                b, a[i], acc[i][jn], FX, FDY, 0, 127, 0, 127);
        }
      }
      if constexpr (WB) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          accb[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              ones, a[i], accb[i], FX, FDY, 0, 127, 0, 127);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      ow0 = own; oh0 = ohn; n0 = nn; pin0 = pinn;
      advance(nn, pinn, ohn, own);
    }
  };
  if (wc == 0) {
    if (bwave) main_loop(std::integral_constant<int, 0>{}, std::true_type{});
    else main_loop(std::integral_constant<int, 0>{}, std::false_type{});
  } else {
    main_loop(std::integral_constant<int, 1>{}, std::false_type{});
  }

  // dequantise into the slice: 1 / (s_X s_dY); bias 1 / s_dY
  const float sdv = fp8_scale(sdys, hist, fmax_dy);
  const float alpha = 1.f / (sdv * fp8_scale(sxs, hist, fmax_x));
  const long long sbase = (long long)split * g.OC;
#pragma unroll
  for (int jn = 0; jn < NJW; ++jn) {
    const int jg = wc * NJW + jn;
    if (jg >= NJ) continue;
    const int tl = jg / NP, pl_ = jg - (jg / NP) * NP;
    const int khg = kh0 + tl / KW, kwl = tl - (tl / KW) * KW;
    const int ng = (khg * g.KW + kwl) * g.Cg + cc * 16 * NP + pl_ * 16 + fg * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int mg = coff_y + mrow0 + i * 16 + fr;
      *(float4*)(ws + (sbase + mg) * g.KK + ng) =
          make_float4(acc[i][jn][0] * alpha, acc[i][jn][1] * alpha,
                      acc[i][jn][2] * alpha, acc[i][jn][3] * alpha);
    }
  }
  if (bwave && fg == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
      wsb[sbase + coff_y + mrow0 + i * 16 + fr] = accb[i][0] / sdv;
  }
}

struct Plan {
  int var;        // 0: unsupported
  int MT, NP, KHT, PB;
  int tiles, mtiles, cchunks, kgroups;
  int splits, kspan;
  HaloGeom g;
};

constexpr int kSlots = 512;   // workgroups resident at two per CU
// bf16 window row pitch Wp = OW + pad (hvk_halo_pitch_pad; at least
// KW - 1).  8 keeps Wp = OW (mod 8): conflict-free transposed reads across
// row wraps.  The tight pitch (2: Wp = OW + KW - 1) moves fewer window
// bytes - the DMA issue, not the LDS, bounds this loop - and measured
// +0.1-1.3 % on AlexNet conv2-5, +3.5 % on VGG conv4_2 / conv5_2, results
// bit-identical (profiles/r6/ab_wgrad_halo_pitch_r6cc.log)
int g_halo_pad = 2;

// fp8: 1-byte elements, 128-pixel steps, 16-B slots (Wp = OW + 16) and the
// fp8 candidate list
Plan make_plan(int N, int H, int W, int C, int OC, int KH, int KW, int pt,
               int pl, int OH, int OW, int groups, int splits,
               bool fp8 = false) {
  const int STEP = fp8 ? 128 : 64, SLOT = fp8 ? 16 : 32, ES = fp8 ? 1 : 2;
  Plan p{};
  const int Cg = C / groups, OCg = OC / groups;
  HaloGeom& g = p.g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.OC = OC;
  g.Cg = Cg; g.OCg = OCg; g.KH = KH; g.KW = KW; g.pt = pt; g.pl = pl;
  g.P = N * OH * OW;
  g.KK = KH * KW * Cg;
  g.Wp = OW + (fp8 ? 16 : std::max(g_halo_pad, KW - 1));
  g.fOW = make_fastdiv(OW);
  if (OH * OW < STEP || KW > 9 || C % 16 != 0 || OC % 16 != 0) return p;
  if ((long long)N * H * W * C * ES >= kBufMaxBytes ||
      (long long)g.P * OC * ES >= kBufMaxBytes)
    return p;
  g.OHW = OH * OW;
  g.fWp = make_fastdiv(g.Wp);
  const int span = (OW - 1 + STEP - 1) / OW + 1;   // output rows of a step
  // with OH * OW a multiple of the step no step crosses an image (steps
  // start at multiples of it): no second image's rows in the window
  const int cross = (OH * OW) % STEP != 0 ? 2 : 1;
  // segment window: slots a kh segment needs, over the image-aligned steps
  // (the last pixel's distance from the first, plus the kw halo)
  const int spi = (g.OHW + STEP - 1) / STEP;
  int dmax = 0;
  for (int st = 0; st < spi; ++st) {
    const int pin = STEP * st, last = min(pin + STEP - 1, g.OHW - 1);
    const int d = (last / OW - pin / OW) * g.Wp + last % OW - pin % OW;
    dmax = max(dmax, d);
  }
  struct Cand { int var, MT, NP, KHT, KW, PB, seg; };
  // in order of preference (the first that fits is taken)
  const Cand cands16[] = {
      {1, 128, 2, 3, 3, 7168, 0},    // AlexNet conv3 / conv5, VGG 14-wide
      {5, 128, 2, 3, 3, 7168, 1},    // VGG 56 / 112-wide (segments)
      {4, 128, 2, 3, 3, 10240, 0},   // VGG 28-wide
      {2, 96, 2, 3, 3, 7168, 0},     // AlexNet conv4
      {7, 96, 3, 3, 3, 8192, 1},     // AlexNet conv1 (space-to-depth)
      {6, 64, 4, 3, 3, 7168, 1},     // VGG conv1_2 (224-wide, 64 channels)
      {3, 128, 3, 1, 5, 5120, 0},    // AlexNet conv2 (5 x 5)
  };
  const Cand cands8[] = {
      {101, 128, 2, 3, 3, 9216, 0},  // VGG 14 / 28 / 56-wide, AlexNet 13
      {102, 128, 2, 3, 3, 7168, 1},  // VGG 112-wide (segments)
      {103, 64, 4, 3, 3, 7168, 1},   // VGG conv1_2 (224-wide, 64 channels)
  };
  const Cand* cands = fp8 ? cands8 : cands16;
  const int ncand = fp8 ? 3 : 7;
  for (int ci = 0; ci < ncand; ++ci) {
    const Cand& c = cands[ci];
    if (KW != c.KW || KH % c.KHT || OCg % c.MT || Cg % (16 * c.NP)) continue;
    if (c.seg) {
      // image-aligned steps waste the tail of each image's last step
      if (spi * STEP * 100 > g.OHW * 103) continue;
      const int segp = dmax + KW;
      if (c.KHT * segp * SLOT > c.PB) continue;
      g.SEGP = segp;
      g.spi = spi;
      g.WR = 0;
    } else {
      const int WR = span + cross * (c.KHT - 1);
      if (WR * g.Wp * SLOT > c.PB) continue;
      g.WR = WR;
      g.SEGP = 0;
      g.spi = 0;
    }
    p.var = c.var; p.MT = c.MT; p.NP = c.NP; p.KHT = c.KHT; p.PB = c.PB;
    break;
  }
  if (!p.var) return p;
  p.mtiles = OCg / p.MT;
  p.cchunks = Cg / (16 * p.NP);
  p.kgroups = KH / p.KHT;
  p.tiles = groups * p.mtiles * p.cchunks * p.kgroups;
  // step units: 64 pixels (full-row window: kspan in pixels), image-aligned
  // steps (segment window: kspan in steps)
  const bool seg = g.SEGP > 0;
  const int steps = seg ? N * spi : (g.P + STEP - 1) / STEP;
  // at most one round of workgroups: a 513th workgroup would run alone in
  // a second round (AlexNet at ceil(512 / tiles) splits: 0.7-0.9x)
  int s = splits > 0 ? splits : kSlots / p.tiles;
  s = max(1, min(s, steps));
  const int ks = (steps + s - 1) / s;
  p.kspan = seg ? ks : ks * STEP;
  p.splits = (steps + ks - 1) / ks;   // every split non-empty
  return p;
}

}  // namespace

static long long finish(float* ws, float* wsb, float* dW, float* dbias, int OC,
                 long long kk, int splits, hipStream_t s);

// Weight gradient through the halo kernel.  ws == nullptr: plan only,
// returns the f32 workspace elements needed ([splits][OC][KK] + [splits]
// [OC]) or -1 when the shape does not take this kernel (the caller uses
// hvk_conv_wgrad).  Else launches the kernel and the finishing pass
// (dW / dbias accumulate) and returns 0, or a HIP error code.
HVK_API long long hvk_conv_wgrad_halo(const void* X, const void* dY, float* dW,
                                      float* dbias, float* ws, int N, int H,
                                      int W, int C, int OC, int KH, int KW,
                                      int pt, int pl, int OH, int OW,
                                      int groups, int splits, hipStream_t s) {
  Plan p = make_plan(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, splits);
  if (!p.var) return -1;
  const long long kk = (long long)KH * KW * (C / groups);
  const long long need = (long long)p.splits * OC * kk + (long long)p.splits * OC;
  if (ws == nullptr) return need;
  if (((uintptr_t)X & 15) || ((uintptr_t)dY & 15)) return -1;
  float* wsb = ws + (long long)p.splits * OC * kk;
  dim3 grid((unsigned)(p.tiles * p.splits)), blk(256);
  const int bias = dbias != nullptr;
  const uint16_t* x = (const uint16_t*)X;
  const uint16_t* dy = (const uint16_t*)dY;
#define HALO_GO(MT, NP, KHT, KW, NJW, PB, SEG)                                \
  hipLaunchKernelGGL((wgrad_halo_kernel<MT, NP, KHT, KW, NJW, PB, SEG>), grid, \
                     blk, 0, s, x, dy, ws, wsb, p.g, p.mtiles, p.cchunks,      \
                     p.kgroups, p.tiles, p.kspan, bias)
  switch (p.var) {
    case 1: HALO_GO(128, 2, 3, 3, 9, 7168, false); break;
    case 2: HALO_GO(96, 2, 3, 3, 9, 7168, false); break;
    case 3: HALO_GO(128, 3, 1, 5, 8, 5120, false); break;
    case 4: HALO_GO(128, 2, 3, 3, 9, 10240, false); break;
    case 5: HALO_GO(128, 2, 3, 3, 9, 7168, true); break;
    case 6: HALO_GO(64, 4, 3, 3, 18, 7168, true); break;
    case 7: HALO_GO(96, 3, 3, 3, 14, 8192, true); break;
    default: return -1;
  }
#undef HALO_GO
  hipError_t e = launch_status(s);
  if (e != hipSuccess) return (long long)e;
  return finish(ws, wsb, dW, dbias, OC, kk, p.splits, s);
}

static long long finish(float* ws, float* wsb, float* dW, float* dbias, int OC,
                 long long kk, int splits, hipStream_t s) {
  const long long n4 = (long long)OC * kk / 4;
  // threads per element: enough workgroups for the chip, <= 32 splits each
  const int R = (splits >= 64 && n4 < (1 << 17)) ? 16
              : (splits >= 16 && n4 < (1 << 19)) ? 4 : 1;
  const int epb = 256 / R;
  const int nmain = (int)((n4 + epb - 1) / epb);
  const int nb = dbias ? (OC + epb - 1) / epb : 0;
  auto fk = R == 16 ? wgrad_finish_kernel<16>
          : R == 4 ? wgrad_finish_kernel<4> : wgrad_finish_kernel<1>;
  hipLaunchKernelGGL(fk, dim3(nmain + nb), dim3(256), 0, s, ws, dW, n4,
                     splits, wsb, dbias, OC, nmain);
  return (long long)launch_status(s);
}

// bf16 window row pitch pad (2 default; see g_halo_pad)
HVK_API void hvk_halo_pitch_pad(int p) { g_halo_pad = p; }

// the plan's split count (tests / autotune logging)
HVK_API int hvk_conv_wgrad_halo_splits(int N, int H, int W, int C, int OC,
                                       int KH, int KW, int pt, int pl, int OH,
                                       int OW, int groups, int splits) {
  Plan p = make_plan(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, splits);
  return p.var ? p.splits : -1;
}

// fp8 weight gradient through the halo kernel (wgrad_halo8_kernel) from the
// e4m3 / e5m2 copies X8 / dY8 (formats fx / fdy: 0 e4m3, 1 e5m2) and their
// scaler states (the hvk_conv_wgrad_fp8 arguments).  ws == nullptr: plan
// only (workspace floats, or -1: use hvk_conv_wgrad_fp8).
HVK_API long long hvk_conv_wgrad_halo_fp8(
    const void* X8, const void* dY8, float* dW, float* dbias, float* ws,
    int N, int H, int W, int C, int OC, int KH, int KW, int pt, int pl,
    int OH, int OW, int groups, int splits, int fx, int fdy, const float* sxs,
    const float* sdys, int hist, float fmax_x, float fmax_dy, hipStream_t s) {
  Plan p = make_plan(N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, splits,
                     true);
  if (!p.var || (fx != 0 && fx != 1) || (fdy != 0 && fdy != 1)) return -1;
  const long long kk = (long long)KH * KW * (C / groups);
  const long long need = (long long)p.splits * OC * kk + (long long)p.splits * OC;
  if (ws == nullptr) return need;
  if (((uintptr_t)X8 & 15) || ((uintptr_t)dY8 & 15)) return -1;
  float* wsb = ws + (long long)p.splits * OC * kk;
  dim3 grid((unsigned)(p.tiles * p.splits)), blk(256);
  const int bias = dbias != nullptr;
  const uint8_t* x = (const uint8_t*)X8;
  const uint8_t* dy = (const uint8_t*)dY8;
#define HALO8_GO(MT, NP, KHT, KW, NJW, PB, SEG, FX, FDY)                       \
  hipLaunchKernelGGL(                                                          \
      (wgrad_halo8_kernel<MT, NP, KHT, KW, NJW, PB, SEG, FX, FDY>), grid, blk, \
      0, s, x, dy, ws, wsb, p.g, p.mtiles, p.cchunks, p.kgroups, p.tiles,      \
      p.kspan, bias, sxs, sdys, hist, fmax_x, fmax_dy)
#define HALO8_FMT(MT, NP, KHT, KW, NJW, PB, SEG)                               \
  if (fx == 0 && fdy == 1) HALO8_GO(MT, NP, KHT, KW, NJW, PB, SEG, 0, 1);     \
  else if (fx == 0 && fdy == 0) HALO8_GO(MT, NP, KHT, KW, NJW, PB, SEG, 0, 0); \
  else if (fx == 1 && fdy == 1) HALO8_GO(MT, NP, KHT, KW, NJW, PB, SEG, 1, 1); \
  else HALO8_GO(MT, NP, KHT, KW, NJW, PB, SEG, 1, 0)
  switch (p.var) {
    case 101: HALO8_FMT(128, 2, 3, 3, 9, 9216, false); break;
    case 102: HALO8_FMT(128, 2, 3, 3, 9, 7168, true); break;
    case 103: HALO8_FMT(64, 4, 3, 3, 18, 7168, true); break;
    default: return -1;
  }
#undef HALO8_FMT
#undef HALO8_GO
  hipError_t e = launch_status(s);
  if (e != hipSuccess) return (long long)e;
  return finish(ws, wsb, dW, dbias, OC, kk, p.splits, s);
}
