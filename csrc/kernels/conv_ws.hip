// conv_ws.hip - weight-stationary stride-1 convolution forward / backward-
// data for layers whose whole filter bank fits in the waves' VGPRs
// (AlexNet conv1 (space-to-depth) and conv2 forward, VGG-16 conv1_2
// forward and backward-data).
//
// Why (round 5): these are the convolutions with a short output dimension
// (48-128 channels per group): the implicit GEMM (gemm_core.h, T4) re-reads
// an im2col tile of the input for every 32-64 deep K step and runs them at
// 24-33 % MFMA (profiles/r4/pmc_mix_alexnet_b2048_r4h.md: conv1 halo kernel
// 24 %, conv2 forward 33 %).  Here:
//   * every wave loads ITS slice of the filter bank (its n-tiles x every K
//     slice, as MFMA B fragments) into VGPRs ONCE (one wave per SIMD, up to
//     ~300 VGPRs of weights) - the weights never touch LDS again;
//   * the workgroups are persistent (one per CU) and walk 64-pixel output
//     tiles; per tile only the input WINDOW those 64 pixels touch (the rows
//     they span + the kh halo, all columns + the kw halo, all channels of
//     the group) is DMA'd into LDS, double buffered, one tile ahead;
//   * every tap's A fragments are ds_read_b128s of that window at a per-
//     lane offset (kh * KP + kw slots).  A slot holds one pixel's CG
//     channels contiguously (what the DMA reads: whole 96-B pixel runs
//     instead of 32-B plane pieces, ~1/3 of the cache lines per byte), padded
//     to 6 / 10 / 14 (mod 16) 16-B chunks so that a ds_read_b128 lane group
//     (16 consecutive pixels, two chunks) hits 16 distinct bank groups;
//     Wp = OW + 16 keeps consecutive pixels in consecutive slots mod 16
//     across row wraps;
//   * the f32 tile goes through LDS (double buffered) to a coalesced
//     epilogue: bias, activation, derivative of the layer below, bf16.
// Per tile the LDS traffic is the window (~40 KiB) against 64 x N x K MACs:
// conv2 forward ~6x fewer operand bytes per FLOP than the T4 loop.
//
// Backward-data (stride 1) is the same kernel: dX = conv(dY, W') with W'
// the flipped, transposed filter bank (read from the dgrad permutation
// wt[g][c][kh][kw][oc] at (KH-1-kh, KW-1-kw)) and the window origin
// KH-1-pt / KW-1-pl.
//
// Window forms (as wgrad_halo.hip): full rows with steps that may span two
// images (narrow images), or per-kh segments with image-aligned tiles (wide
// images: VGG 224).
#include "conv_geom.h"

// diagnostic builds only (wrong results by design): 1 no window DMA, 2 no
// epilogue stores, 4 no MFMAs
#ifndef HVK_WS_ABL
#define HVK_WS_ABL 0
#endif

using namespace hvk;

namespace {

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8;
typedef __attribute__((address_space(3))) f32x4 lds_f4;

struct WsGeom {
  int N, H, W, C;          // window source (x or dY), NHWC, C channels total
  int OH, OW;              // output pixels
  int OCT, OCg;            // output channels: total, per group
  int pt, pl;              // input row = oh + kh - pt, column = ow + kw - pl
  int P, OHW;
  int Wp, WR, SEGP, spi, PB;   // PB: window bytes
  int pairs, wpp, tiles;   // (group, n-tile) pairs, WGs per pair, tiles
  FastDiv fOW, fWp, fOHW, fSPI;
};

// CG: source channels per group, KH x KW taps, NJW
// n-tiles per wave, WM x WN waves, TM m-tiles per pixel tile (TM * 16
// pixels; MI = TM / WM per wave), SEG: segment window, FLIP: backward-data
// weights
// 16-B chunks per window slot: CG / 8, padded to 6, 10 or 14 mod 16
__host__ __device__ constexpr int ws_cps(int cg) {
  return (cg / 8) % 16 == 6 || (cg / 8) % 16 == 10 || (cg / 8) % 16 == 14
             ? cg / 8
             : ws_cps(cg + 8);
}

template <int CG, int KH, int KW, int NJW, int WM, int WN, int TM, bool SEG,
          bool FLIP, int NBW>
__global__ void __launch_bounds__(256, 1)
__attribute__((amdgpu_waves_per_eu(1, 1)))
conv_ws_kernel(const uint16_t* __restrict__ src,
               const uint16_t* __restrict__ wts, const float* __restrict__ bias,
               uint16_t* __restrict__ out, const uint16_t* __restrict__ aux,
               int act, int aux_act, WsGeom g) {
  constexpr int K = KH * KW * CG;
  constexpr int NSL = (K + 31) / 32;
  constexpr int MI = TM / WM;
  constexpr int TPX = TM * 16;               // pixels per tile
  constexpr int NOUT = WN * NJW * 16;
  static_assert(WM * WN == 4 && MI * WM == TM, "four waves");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  lds_u8* sm = (lds_u8*)smem;
  constexpr int CPS = ws_cps(CG);            // 16-B chunks per slot
  constexpr int SB = CPS * 16;                // slot bytes
  // one window stage, rounded up to whole 1-KiB DMA pieces (the last
  // piece's out-of-window lanes write zeros inside the stage)
  const int WS = SEG ? KH * g.SEGP : g.WR * g.Wp;
  const int WIN = (WS * SB + 1023) / 1024 * 1024;

  const int pair = blockIdx.x % g.pairs;
  const int widx = blockIdx.x / g.pairs;
  const int nt = pair % (g.OCg / NOUT);
  const int gi = pair / (g.OCg / NOUT);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w % WM, wn = w / WM;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- the wave's filter slice in VGPRs: B fragments (row n = output
  // channel, 8 consecutive k of chunk fq) for n-tiles j, K slices s
  bf16x8 wreg[NJW][NSL];
  {
    const long long obase = (long long)gi * g.OCg + nt * NOUT;
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const long long row = obase + (wn * NJW + j) * 16 + fr;
#pragma unroll
      for (int s = 0; s < NSL; ++s) {
        const int k = s * 32 + fq * 8;
        bf16x8 v = {};
        if (k < K) {
          const int tap = k / CG, c = k - (k / CG) * CG;
          int kh = tap / KW, kw = tap - (tap / KW) * KW;
          if (FLIP) { kh = KH - 1 - kh; kw = KW - 1 - kw; }
          v = *(const bf16x8*)(wts + row * K + (kh * KW + kw) * CG + c);
        }
        wreg[j][s] = v;
      }
    }
  }
  // every weight load done before the tile loop: the compiler's waits for
  // them would otherwise sit inside the MFMA stream, where vmcnt (loads,
  // stores and LDS-DMA retire in order) also waits for the next tile's
  // window DMA.  A real s_waitcnt (not inline asm) so that the waitcnt pass
  // sees it: vmcnt(0), expcnt / lgkmcnt left at their maxima
  __builtin_amdgcn_s_waitcnt(0x0F70);
  // ---- the bias of this lane's output channels (constant per workgroup)
  float4 bsv[NJW];
#pragma unroll
  for (int j = 0; j < NJW; ++j) {
    const int oc = gi * g.OCg + nt * NOUT + (wn * NJW + j) * 16 + fq * 4;
    bsv[j] = bias ? *(const float4*)(bias + oc) : make_float4(0.f, 0.f, 0.f,
                                                              0.f);
  }
  // ---- per-lane window offsets of each K slice (chunk fq of slice s):
  // tap (kh, kw), plane, 16-B half; K padding reads slot 0 (zero weights)
  const int KP = SEG ? g.SEGP : g.Wp;
  uint32_t ofs[NSL];
#pragma unroll
  for (int s = 0; s < NSL; ++s) {
    const int k = s * 32 + fq * 8;
    uint32_t o = 0;
    if (k < K) {
      const int tap = k / CG, c = k - (k / CG) * CG;
      const int kh = tap / KW, kw = tap - (tap / KW) * KW;
      o = (uint32_t)((kh * KP + kw) * SB + (c >> 3) * 16);
    }
    ofs[s] = o;
  }

  // ---- window DMA slots (lane-linear 1-KiB pieces)
  const __amdgpu_buffer_rsrc_t rsrc = dma_rsrc(src);
  const int NB = WIN / 1024;
  const uint32_t rowbytes = (uint32_t)g.W * g.C * 2u;
  const uint32_t pixbytes = (uint32_t)g.C * 2u;
  const int coff = gi * CG;
  // tile decode: first pixel's image, in-image index, row, column
  auto decode = [&](int tl, int& n, int& pin, int& oh, int& ow) {
    if constexpr (SEG) {
      n = (int)fdiv((uint32_t)tl, g.fSPI);
      pin = (tl - n * g.spi) * TPX;
    } else {
      const int p = tl * TPX;
      n = (int)fdiv((uint32_t)p, g.fOHW);
      pin = p - n * g.OHW;
    }
    oh = (int)fdiv((uint32_t)pin, g.fOW);
    ow = pin - oh * g.OW;
  };
  // per-lane DMA slot geometry of each of this wave's pieces (pieces w,
  // w + 4, ...), precomputed once: window row (or kh segment) | column (or
  // segment slot) << 16, and the channel byte offset | valid << 31
  // packed: row / segment (8 bits) | column / slot << 8 (12 bits) | channel
  // bytes << 20 (11 bits) | valid << 31
  uint32_t pgeo[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int pi = w + 4 * i;
    const int q = pi * 64 + lane;            // 16-B chunk of the stage
    const int slot = q / CPS, ch = q - (q / CPS) * CPS;
    const int kp = SEG ? g.SEGP : g.Wp;
    const int r = slot / kp, cl = slot - r * kp;
    bool ok = pi < NB && slot < WS && ch * 8 < CG;
    if constexpr (!SEG) ok = ok && cl < g.OW + KW - 1;
    pgeo[i] = (uint32_t)r | ((uint32_t)cl << 8) |
              ((uint32_t)(coff + ch * 8) * 2u << 20) |
              (ok ? 0x80000000u : 0u);
  }
  auto issue = [&](int tl, int stage) {
    if constexpr ((HVK_WS_ABL & 1) != 0) return;
    int n, pin, oh, ow;
    decode(tl, n, pin, oh, ow);
    uint8_t* dst = smem + stage * WIN;
    const int rc = g.OH - oh + KH - 1;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (w + 4 * i >= NB) break;   // wave-uniform
      const int r = (int)(pgeo[i] & 0xffu);
      const int cl = (int)((pgeo[i] >> 8) & 0xfffu);
      bool ok = (pgeo[i] >> 31) != 0;
      int ih, iw, nn = n;
      if constexpr (SEG) {
        const uint32_t sj = (uint32_t)(ow + cl);
        const int rr = (int)fdiv(sj, g.fWp);
        const int col = (int)sj - rr * g.Wp;
        ih = oh + rr + r - g.pt;
        iw = col - g.pl;
        ok = ok && col < g.OW + KW - 1;
      } else {
        iw = cl - g.pl;
        const bool first = r < rc;
        ih = (first ? oh + r : r - rc) - g.pt;
        nn = first ? n : n + 1;
      }
      ok = ok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W &&
           nn < g.N;
      const uint32_t v =
          ok ? ((uint32_t)nn * g.H + (uint32_t)ih) * rowbytes +
                   (uint32_t)iw * pixbytes + ((pgeo[i] >> 20) & 0x7ffu)
             : kBufOOB;
      dma16(rsrc, dst + (w + 4 * i) * 1024, v);
    }
  };

  const int stride = g.wpp;
  int tl = widx;
  if (tl >= g.tiles) return;
  issue(tl, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int m0w = wm * MI * 16;   // first pixel row of this wave's m-tiles
  for (int it = 0; tl < g.tiles; ++it, tl += stride) {
    const int cur = it & 1;
    const int tnext = tl + stride;
    if (tnext < g.tiles) issue(tnext, cur ^ 1);
    int n, pin, oh0, ow0;
    decode(tl, n, pin, oh0, ow0);
    // window slot bases of this lane's pixels (fr of each m-tile)
    uint32_t bb[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int d = m0w + i * 16 + fr;
      const uint32_t owd = (uint32_t)(ow0 + d);
      const uint32_t gr = fdiv(owd, g.fOW);
      const int owr = (int)(owd - gr * (uint32_t)g.OW);
      int slot;
      if constexpr (SEG) {
        slot = pin + d < g.OHW ? (int)gr * g.Wp + owr - ow0 : 0;
      } else {
        slot = ((int)gr + ((oh0 + (int)gr >= g.OH) ? KH - 1 : 0)) * g.Wp + owr;
      }
      bb[i] = (uint32_t)(cur * WIN + slot * SB);
    }
    f32x4 acc[MI][NJW];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software pipeline: the A fragments of slice s + PD are read while
    // slice s's MFMAs run (one wave per SIMD: nothing else hides the LDS
    // latency); scheduling barriers keep the compiler from sinking the
    // reads back next to their MFMAs
    constexpr int PD = 2;
    bf16x8 a[PD + 1][MI];
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[s][i] = *(lds_bf16x8*)(sm + bb[i] + ofs[s]);
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      if (s + PD < NSL) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          a[(s + PD) % (PD + 1)][i] =
              *(lds_bf16x8*)(sm + bb[i] + ofs[s + PD]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((HVK_WS_ABL & 4) == 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                wreg[j][s], a[s % (PD + 1)][i], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          acc[i][0][0] += (float)a[s % (PD + 1)][i][0];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // next window landed; every read of this window done (before the
    // epilogue's stores, which vmcnt would otherwise wait for too)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // direct epilogue from the accumulators (lane: D[n = fq*4 + r][m =
    // fr], 4 consecutive output channels of one pixel): bias, activation,
    // derivative of the layer below, bf16, one 8-B store per tile pair.
    // One workgroup per CU: an LDS-staged epilogue's barrier would idle the
    // matrix cores (nothing else on the CU covers it)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0w + i * 16 + fr;
      long long pg;
      bool ok;
      if constexpr (SEG) {
        ok = pin + m < g.OHW;
        pg = (long long)n * g.OHW + pin + m;
      } else {
        pg = (long long)tl * TPX + m;
        ok = pg < g.P;
      }
      if (!ok || ((HVK_WS_ABL & 2) && acc[i][0][0] != 1234.5f)) continue;
#pragma unroll
      for (int j = 0; j < NJW; ++j) {
        const int oc = gi * g.OCg + nt * NOUT + (wn * NJW + j) * 16 + fq * 4;
        float v[4] = {acc[i][j][0] + bsv[j].x, acc[i][j][1] + bsv[j].y,
                      acc[i][j][2] + bsv[j].z, acc[i][j][3] + bsv[j].w};
        act_fwd_n<4>(v, act);
        const long long oi = pg * g.OCT + oc;
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
  }
}

struct WsPlan {
  int var;     // 0: unsupported
  size_t lds;
  int grid;
  WsGeom g;
};

// one workgroup per CU, at most 160 KiB of LDS
constexpr int kCUs = 256;

WsPlan ws_plan(int N, int H, int W, int C, int OH, int OW, int OCT, int KH,
               int KW, int pt, int pl, int groups, bool dgrad) {
  WsPlan p{};
  WsGeom& g = p.g;
  const int CG = C / groups, OCg = OCT / groups;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.OCT = OCT;
  g.OCg = OCg; g.pt = pt; g.pl = pl;
  g.P = N * OH * OW;
  g.OHW = OH * OW;
  g.Wp = OW + 16;
  g.fOW = make_fastdiv(OW);
  g.fWp = make_fastdiv(g.Wp);
  if (g.OHW < 64 || C % 16 || OCT % 8) return p;
  if ((long long)N * H * W * C * 2 >= kBufMaxBytes) return p;
  struct Cand { int var, CG, KH, KW, NOUT, dgrad, TPX; };
  const Cand cands[] = {
      {1, 48, 5, 5, 128, 0, 64},    // AlexNet conv2 forward
      {2, 48, 3, 3, 96, 0, 128},    // AlexNet conv1 forward (space-to-depth)
      {3, 64, 3, 3, 64, 0, 128},    // VGG-16 conv1_2 forward
      {4, 64, 3, 3, 64, 1, 128},    // VGG-16 conv1_2 backward-data
  };
  const Cand* c = nullptr;
  for (const Cand& k : cands)
    if (k.CG == CG && k.KH == KH && k.KW == KW && OCg % k.NOUT == 0 &&
        k.dgrad == (int)dgrad) {
      c = &k;
      break;
    }
  if (!c) return p;
  const int TPX = c->TPX;
  if (g.OHW < TPX) return p;
  const int span = (OW - 1 + TPX - 1) / OW + 1;
  const int cross = g.OHW % TPX ? 2 : 1;
  const int WR = span + cross * (KH - 1);
  const int spi = (g.OHW + TPX - 1) / TPX;
  int dmax = 0;
  for (int st = 0; st < spi; ++st) {
    const int pin = TPX * st, last = min(pin + TPX - 1, g.OHW - 1);
    dmax = max(dmax, (last / OW - pin / OW) * g.Wp + last % OW - pin % OW);
  }
  const int segp = dmax + KW;
  const int SB = ws_cps(CG) * 16;
  const int full_b = WR * g.Wp * SB, seg_b = KH * segp * SB;
  const bool seg = seg_b < full_b && spi * TPX * 100 <= g.OHW * 103;
  g.PB = seg ? seg_b : full_b;   // window bytes
  g.WR = seg ? 0 : WR;
  g.SEGP = seg ? segp : 0;
  g.spi = seg ? spi : 0;
  p.lds = 2 * (((size_t)g.PB + 1023) / 1024 * 1024);
  if (p.lds > 160 * 1024) return p;
  g.pairs = groups * (OCg / c->NOUT);
  if (g.pairs > kCUs) return p;
  g.wpp = kCUs / g.pairs;
  g.tiles = seg ? N * spi : (g.P + TPX - 1) / TPX;
  g.fOHW = make_fastdiv(g.OHW);
  g.fSPI = make_fastdiv(seg ? spi : 1);
  p.grid = g.pairs * g.wpp;
  p.var = c->var * 2 + (seg ? 1 : 0);
  return p;
}

template <int CG, int KH, int KW, int NJW, int WM, int WN, int TM, bool SEG,
          bool FLIP, int NBW>
hipError_t go_ws(const WsPlan& p, const void* src, const void* wts,
                 const float* bias, void* out, const void* aux, int act,
                 int aux_act, hipStream_t s) {
  // NBW: DMA pieces per wave the plan allows (the window's 1-KiB pieces / 4)
  if ((((size_t)p.g.PB + 1023) / 1024 + 3) / 4 > NBW)
    return hipErrorInvalidValue;
  auto kern = conv_ws_kernel<CG, KH, KW, NJW, WM, WN, TM, SEG, FLIP, NBW>;
  static bool attr = false;   // once per instantiation, before any capture
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(
        (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
        160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)p.grid), dim3(256), p.lds, s,
                     (const uint16_t*)src, (const uint16_t*)wts, bias,
                     (uint16_t*)out, (const uint16_t*)aux, act, aux_act, p.g);
  return launch_status(s);
}

hipError_t ws_launch(const WsPlan& p, const void* src, const void* wts,
                     const float* bias, void* out, const void* aux, int act,
                     int aux_act, hipStream_t s) {
  switch (p.var) {
    case 2: return go_ws<48, 5, 5, 2, 1, 4, 4, false, false, 13>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 3: return go_ws<48, 5, 5, 2, 1, 4, 4, true, false, 13>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 4: return go_ws<48, 3, 3, 3, 2, 2, 8, false, false, 14>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 5: return go_ws<48, 3, 3, 3, 2, 2, 8, true, false, 14>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 6: return go_ws<64, 3, 3, 2, 2, 2, 8, false, false, 18>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 7: return go_ws<64, 3, 3, 2, 2, 2, 8, true, false, 18>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 8: return go_ws<64, 3, 3, 2, 2, 2, 8, false, true, 18>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    case 9: return go_ws<64, 3, 3, 2, 2, 2, 8, true, true, 18>(
        p, src, wts, bias, out, aux, act, aux_act, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// Forward: Y[N][OH][OW][OC] = act(conv(X, W) + bias), stride 1, X bf16 NHWC,
// W [OC][KH][KW][C/g].  Returns 0, -2 when the shape does not take this
// kernel (the caller uses the implicit GEMM), or a HIP error.
HVK_API int hvk_conv_fwd_ws(const void* X, const void* Wt, const float* bias,
                            void* Y, int N, int H, int W, int C, int OC,
                            int KH, int KW, int pt, int pl, int OH, int OW,
                            int groups, int act, hipStream_t s) {
  if (((uintptr_t)X & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)Y & 15))
    return -2;
  WsPlan p = ws_plan(N, H, W, C, OH, OW, OC, KH, KW, pt, pl, groups, false);
  if (!p.var) return -2;
  return (int)ws_launch(p, X, Wt, bias, Y, nullptr, act, 0, s);
}

// Backward-data: dX[N][H][W][C] = conv^T(dY, W) [* act'(aux)], stride 1,
// from the dgrad weight permutation wt[g][c][kh][kw][oc].  -2: not taken.
HVK_API int hvk_conv_dgrad_ws(const void* dY, const void* Wt, void* dX, int N,
                              int H, int W, int C, int OC, int KH, int KW,
                              int pt, int pl, int OH, int OW, int groups,
                              const void* aux, int aux_act, hipStream_t s) {
  if (((uintptr_t)dY & 15) || ((uintptr_t)Wt & 15) || ((uintptr_t)dX & 15) ||
      ((uintptr_t)aux & 15))
    return -2;
  // the window source is dY (OH x OW, OC channels), the output dX (H x W, C
  // channels), origin KH - 1 - pt / KW - 1 - pl
  WsPlan p = ws_plan(N, OH, OW, OC, H, W, C, KH, KW, KH - 1 - pt, KW - 1 - pl,
                     groups, true);
  if (!p.var) return -2;
  return (int)ws_launch(p, dY, Wt, nullptr, dX, aux, 0, aux_act, s);
}
