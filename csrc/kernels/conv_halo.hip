// conv_halo.hip - stride-1 convolution forward / backward-data with the
// input tile held in LDS (the "halo" of a block's output tile).
//
// The implicit GEMM of gemm_core.h re-gathers the A operand (im2col of the
// input) from L2 for every K tile: each input element crosses L2 -> LDS once
// per filter tap (25 times for a 5 x 5 kernel).  For a block of BM output
// pixels forming a TH x TW spatial tile of one image and N up to 128 output
// channels, that is ~0.0156 B/FLOP at 128 x 128 and ~0.031 B/FLOP for the
// 48-wide AlexNet conv2 backward-data - L2-bandwidth bound near the
// 17-19 TB/s an MI355X moves L2 -> LDS (MI355X_MICROARCH.md, "Indexed rows").
// Here the block DMAs its (TH + KH - 1) x (TW + KW - 1) input pixels x the
// group's channels into LDS once, and every K tile's A fragments are read
// from that image at the tap's offset: A traffic drops ~KH*KW / (halo
// overhead) times, and only the weights stream per K tile.
//
// Same GEMM as gemm_core.h's conv kernels - A[m][k], k = (kh, kw, c), B the
// K-major weights (forward: W[oc][kh][kw][c]; backward-data: the permuted
// Wt[c][kh][kw][oc], dY as the halo source with the taps flipped) - and the
// same 16x16x32 MFMA sequence per K tile, so the results are bit-identical to
// the implicit-GEMM kernels.  LDS image of the halo: [pixel][CP chunks of 8
// channels], CP odd so that the 16 rows of a ds_read_b128 fragment land on 16
// distinct bank groups (conflict-free) - filled by buffer LDS-DMA, zeros
// outside the image and in the pad chunk.
#include <algorithm>

#include "gemm_core.h"

namespace {

struct HaloGeom {
  int N, H, W, Ctot, Ch;   // halo source [N][H][W][Ctot], Ch channels / group
  int OH, OW;              // GEMM rows: output pixels
  int KH, KW;
  int oy, ox;              // halo origin = (oh0 + oy, ow0 + ox)
  int flip;                // backward-data: tap (kh, kw) at (KH-1-kh, KW-1-kw)
  int TH, TW, HW_, HP;     // tile, halo width, halo pixels
  int CP;                  // LDS chunks per halo pixel (odd)
  int tiles_x, tiles_sp;   // spatial tiles per row of tiles, per group
  FastDiv fTW, fHW, fCP, fCh, fKW, fTX, fTSP;
};

// EP 2: the register epilogue (as the T4 loop's, gemm_t4.h): the MFMAs
// compute the transposed tile, each lane finishes 4 consecutive output
// channels of one pixel in registers (bias, activation, derivative of the
// layer below, bf16) into a bf16 image of the tile, then whole 16-B chunks
// go out (opt-in, hvk_gemm_variant 54); EP 0 stages the f32 tile
template <int BN_, bool W8, int VAR, int EP = 0>
__global__ void __launch_bounds__(W8 ? 512 : NTHR, 2)
conv_halo_kernel(HaloGeom hg, const uint16_t* __restrict__ src, DenseK lb,
                 Epi epi, int K, int tiles_n) {
  constexpr int NW = W8 ? 8 : 4;
  constexpr int NT = NW * 64;
  constexpr int WNC = VAR == 2 ? 1 : NW / 2;
  constexpr int MT = VAR == 2 ? 2 : 4;
  constexpr int WMR = 16 * MT;
  constexpr int NC = VAR == 2 ? 48 : BN_;
  constexpr int NB = NC / (16 * WNC);
  static_assert((NW / WNC) * WMR == BM && NB * 16 * WNC == NC, "layout");
  constexpr int SB = BN_ * BK;                   // one B stage (elements)
  constexpr int NIB = BN_ / (8 * NW);            // B DMA pieces per wave
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int hsz = ((hg.HP * hg.CP * 8) + 511) / 512 * 512;  // halo elements
  uint16_t* sH = smem;
  uint16_t* sB = smem + hsz;

  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = wgid % tiles_n;
  const int rest = wgid / tiles_n;
  uint32_t gi, sp, img, tsp, ty, tx;
  fdivmod((uint32_t)rest, hg.fTSP, gi, sp);
  // spatial tile sp -> (image, tile row, tile column)
  const int tiles_img = hg.tiles_sp / hg.N;
  img = sp / tiles_img;
  tsp = sp - img * tiles_img;
  fdivmod(tsp, hg.fTX, ty, tx);
  const int oh0 = (int)ty * hg.TH, ow0 = (int)tx * hg.TW;
  lb.group((int)gi);
  const int n0 = tn * NC;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int w = __builtin_amdgcn_readfirstlane(wid);
  const int wm = wid / WNC, wn = wid % WNC;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- halo fill: chunk slot s -> (pixel p, chunk j); zeros off-image
  {
    const __amdgpu_buffer_rsrc_t rs = dma_rsrc(src);
    const int nch = hg.HP * hg.CP;
    const int hy0 = oh0 + hg.oy, hx0 = ow0 + hg.ox;
    const long long ibase = (long long)img * hg.H * hg.W * hg.Ctot +
                            (long long)gi * hg.Ch;
    for (int s0 = w * 64; s0 < nch; s0 += NW * 64) {
      const int s = s0 + lane;
      uint32_t p, j, hy, hx;
      fdivmod((uint32_t)s, hg.fCP, p, j);
      fdivmod(p, hg.fHW, hy, hx);
      const int ih = hy0 + (int)hy, iw = hx0 + (int)hx;
      const bool ok = s < nch && (int)j * 8 < hg.Ch &&
                      (unsigned)ih < (unsigned)hg.H &&
                      (unsigned)iw < (unsigned)hg.W;
      const long long e = ibase + ((long long)ih * hg.W + iw) * hg.Ctot +
                          (long long)j * 8;
      dma16(rs, sH + s0 * 8, ok ? (uint32_t)(e * 2) : kBufOOB);
    }
  }
  // ---- B (weights, K-major) stages: the gemm_core.h DenseK DMA pieces
  const __amdgpu_buffer_rsrc_t rb = dma_rsrc(lb.dbase());
  const int kc = 8 * ((lane & 7) ^ ((lane >> 3) & 7));
  uint32_t vb[NIB];
#pragma unroll
  for (int i = 0; i < NIB; ++i)
    vb[i] = lb.row_voff(n0 + 8 * (w * NIB + i) + (lane >> 3));
  auto issue_b = [&](int k0, uint16_t* dst) {
    const bool kin = k0 + kc < lb.K;
    const uint32_t kbyte = 2u * (uint32_t)(k0 + kc);
#pragma unroll
    for (int i = 0; i < NIB; ++i)
      dma16(rb, dst + (w * NIB + i) * 512, kin ? vb[i] + kbyte : kBufOOB);
  };

  // per m-tile: the row's halo pixel (tile-local (py, px) -> py*HW_ + px)
  int hpix[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = wm * WMR + i * 16 + fr;
    uint32_t py, px;
    fdivmod((uint32_t)m, hg.fTW, py, px);
    hpix[i] = m < hg.TH * hg.TW ? (int)py * hg.HW_ + (int)px : 0;
  }
  f32x4 acc[MT][NB];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto frag_b = [&](const uint16_t* s, int rowbase, int ks) -> bf16x8 {
    int row = rowbase + fr;
    int c = ks * 4 + fq;
    return *(const bf16x8*)(s + row * 64 + ((c ^ (row & 7)) << 3));
  };
  // the lane's k chunk (k0 + 32 ks + 8 fq) -> halo offset of its tap and
  // chunk; k past K reads tap 0 (finite data; its B is zero)
  auto koff = [&](int k) -> int {
    uint32_t tp, c, kh, kw;
    fdivmod((uint32_t)(k < K ? k : 0), hg.fCh, tp, c);
    fdivmod(tp, hg.fKW, kh, kw);
    if (hg.flip) {
      kh = hg.KH - 1 - kh;
      kw = hg.KW - 1 - kw;
    }
    return ((int)kh * hg.HW_ + (int)kw) * hg.CP + (int)(c >> 3);
  };
  auto compute = [&](int k0, const uint16_t* sBc) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ko = koff(k0 + ks * 32 + fq * 8);
      bf16x8 af[MT], bfv[NB];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *(const bf16x8*)(sH + (hpix[i] * hg.CP + ko) * 8);
#pragma unroll
      for (int j = 0; j < NB; ++j)
        bfv[j] = frag_b(sBc, wn * (NC / WNC) + j * 16, ks);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (EP == 2)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                bfv[j], af[i], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                af[i], bfv[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  const int nk = (K + BK - 1) / BK;
  issue_b(0, sB);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue_b((kt + 1) * BK, sB + (cur ^ 1) * SB);
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(kt * BK, sB + cur * SB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  if constexpr (EP == 2) {
    constexpr int LDO = NC + 8;
    static_assert(BM * LDO * 2 <= 80 * 1024, "bf16 tile fits");
    uint16_t* sO = smem;
    const int rows = hg.TH * hg.TW;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int ml = wm * WMR + i * 16 + fr;     // tile pixel of this lane
      uint32_t py, px;
      fdivmod((uint32_t)ml, hg.fTW, py, px);
      const int oh = oh0 + (int)py, ow = ow0 + (int)px;
      const bool pin = ml < rows && oh < hg.OH && ow < hg.OW;
      const int P = ((int)img * hg.OH + oh) * hg.OW + ow;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int nl = wn * (NC / WNC) + j * 16 + fq * 4;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        uint2 o = make_uint2(0u, 0u);
        if (pin && n0 + nl < epi.N) o = epi.pre4((int)gi, P, n0 + nl, v);
        *(uint2*)(sO + ml * LDO + nl) = o;
      }
    }
    __syncthreads();
    constexpr int CH = NC / 8;
    const float qs = epi.q8.q ? fp8_scale(epi.q8.st, epi.q8.hist, epi.q8.fmax)
                              : 1.f;
    float amax = 0.f;
    for (int q = t; q < rows * CH; q += NT) {
      const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
      uint32_t py, px;
      fdivmod((uint32_t)row, hg.fTW, py, px);
      const int oh = oh0 + (int)py, ow = ow0 + (int)px;
      if (oh >= hg.OH || ow >= hg.OW || n0 + c8 >= epi.N) continue;
      const int P = ((int)img * hg.OH + oh) * hg.OW + ow;
      const uint4 ob = *(const uint4*)(sO + row * LDO + c8);
      const long long idx = (long long)(P + (int)gi * epi.grow) * epi.ldc +
                            n0 + c8 + (int)gi * epi.gcol;
      *(uint4*)((uint16_t*)epi.c + idx) = ob;
      if (epi.q8.q) q8_store8(epi.q8, idx, ob, qs, amax);
    }
    if (epi.q8.q) {  // block-uniform
      __syncthreads();
      q8_block_amax(epi.q8, amax, (float*)smem);
    }
    return;
  }
  // ---- epilogue: f32 tile through LDS, then row-contiguous stores of the
  // tile's in-image pixels
  constexpr int LDC = BN_ + 4;
  float* sC = (float*)smem;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int rb2 = wm * WMR + i * 16 + fq * 4;
      int cc = wn * (NC / WNC) + j * 16 + fr;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sC[(rb2 + rr) * LDC + cc] = acc[i][j][rr];
    }
  __syncthreads();
  constexpr int CH = NC / 8;
  const bool fast = epi.fast_ok();
  const int rows = hg.TH * hg.TW;
  const float qs = epi.q8.q ? fp8_scale(epi.q8.st, epi.q8.hist, epi.q8.fmax)
                            : 1.f;
  float amax = 0.f;
  for (int q = t; q < rows * CH; q += NT) {
    const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
    uint32_t py, px;
    fdivmod((uint32_t)row, hg.fTW, py, px);
    const int oh = oh0 + (int)py, ow = ow0 + (int)px;
    if (oh >= hg.OH || ow >= hg.OW) continue;
    const int P = ((int)img * hg.OH + oh) * hg.OW + ow;
    const float4* sp4 = (const float4*)(sC + row * LDC + c8);
    float v[8];
    const float4 lo = sp4[0], hi = sp4[1];
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    if (fast && n0 + c8 + 8 <= epi.N)
      epi.store8_fast((int)gi, P, n0 + c8, v, qs, &amax);
    else
      epi.store8((int)gi, P, n0 + c8, v);
  }
  if (epi.q8.q) {  // block-uniform
    __syncthreads();
    q8_block_amax(epi.q8, amax, sC);
  }
}

// Tile choice: the TH x TW (<= 128 pixels) that wastes the fewest GEMM rows
// over the OH x OW image, ties to the squarer halo.
void pick_tile(int OH, int OW, int KH, int KW, int& TH, int& TW) {
  long long best = -1;
  double bestw = 0;
  for (int th = 1; th <= 128 && th <= OH + 7; ++th) {
    const int tw = std::min(128 / th, OW);
    if (tw < 1) break;
    const long long tiles = (long long)((OH + th - 1) / th) * ((OW + tw - 1) / tw);
    const double eff = (double)OH * OW / (tiles * 128.0);
    const long long halo = (long long)(th + KH - 1) * (tw + KW - 1);
    const double score = eff - 1e-6 * halo;
    if (best < 0 || score > bestw) {
      best = tiles;
      bestw = score;
      TH = th;
      TW = tw;
    }
  }
}

HaloGeom make_halo(int N, int H, int W, int Ctot, int Ch, int OH, int OW,
                   int KH, int KW, int oy, int ox, int flip) {
  HaloGeom g;
  g.N = N; g.H = H; g.W = W; g.Ctot = Ctot; g.Ch = Ch;
  g.OH = OH; g.OW = OW; g.KH = KH; g.KW = KW; g.oy = oy; g.ox = ox;
  g.flip = flip;
  pick_tile(OH, OW, KH, KW, g.TH, g.TW);
  g.HW_ = g.TW + KW - 1;
  g.HP = (g.TH + KH - 1) * g.HW_;
  g.CP = (Ch / 8) | 1;
  g.tiles_x = (OW + g.TW - 1) / g.TW;
  g.tiles_sp = N * ((OH + g.TH - 1) / g.TH) * g.tiles_x;
  g.fTW = make_fastdiv(g.TW); g.fHW = make_fastdiv(g.HW_);
  g.fCP = make_fastdiv(g.CP); g.fCh = make_fastdiv(Ch);
  g.fKW = make_fastdiv(KW); g.fTX = make_fastdiv(g.tiles_x);
  g.fTSP = make_fastdiv(g.tiles_sp);
  return g;
}

// LDS bytes of a launch: halo + 2 B stages, or the f32 C tile if larger
size_t halo_lds(const HaloGeom& g, int bn) {
  const size_t hsz = ((size_t)g.HP * g.CP * 8 + 511) / 512 * 512 * 2;
  const size_t ops = hsz + 2 * (size_t)bn * BK * 2;
  const size_t ctile = (size_t)BM * (bn + 4) * 4;
  return std::max(ops, ctile);
}

template <int BN_, bool W8, int VAR, int EP>
hipError_t launch_halo_(const HaloGeom& g, const uint16_t* src,
                        const DenseK& lb, const Epi& e, int K, int N,
                        int groups, hipStream_t s) {
  const int tiles_n = (N + (VAR == 2 ? 48 : BN_) - 1) / (VAR == 2 ? 48 : BN_);
  const size_t lds = halo_lds(g, BN_);
  auto kern = conv_halo_kernel<BN_, W8, VAR, EP>;
  static bool attr = false;  // once per instantiation, before any capture
  if (!attr) {
    hipError_t err = hipFuncSetAttribute(
        (const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
        80 * 1024);
    if (err != hipSuccess) return err;
    attr = true;
  }
  const long long grid = (long long)tiles_n * g.tiles_sp * groups;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(W8 ? 512 : NTHR), lds, s,
                     g, src, lb, e, K, tiles_n);
  return launch_status(s);
}

// the register epilogue where the output takes it (bf16, written once,
// 8-column groups: Epi::pre4) - opt-in (hvk_gemm_variant 54): AlexNet conv1
// measured 536 -> 491 TF with it
template <int BN_, bool W8, int VAR>
hipError_t launch_halo(const HaloGeom& g, const uint16_t* src, const DenseK& lb,
                       const Epi& e, int K, int N, int groups, hipStream_t s) {
  if (hvk_gemm_variant == 54 && e.fast_ok() && !e.out_f32 && e.beta == 0.f &&
      e.ones_col < 0 && (e.N & 7) == 0)
    return launch_halo_<BN_, W8, VAR, 2>(g, src, lb, e, K, N, groups, s);
  return launch_halo_<BN_, W8, VAR, 0>(g, src, lb, e, K, N, groups, s);
}

// the halo path applies: stride 1, 16-B channel chunks, a halo that fits LDS
// beside two B stages at 2 workgroups per CU (<= 80 KiB), 32-bit offsets,
// and spatial tiles that fill >= 85 % of the 128 GEMM rows (a 13 x 13 image
// fills 66 %: the implicit GEMM, which packs rows across images, wins there)
bool halo_ok(const HaloGeom& g, int bn, const void* src, const void* wt) {
  const double fill = (double)g.OH * g.OW * g.N / ((double)g.tiles_sp * BM);
  return g.Ch % 8 == 0 && g.Ctot % 8 == 0 && al16(src) && al16(wt) &&
         halo_lds(g, bn) <= 80 * 1024 && fill >= 0.85 &&
         (long long)g.N * g.H * g.W * g.Ctot * 2 < kBufMaxBytes;
}

// the GEMM column tile for N output channels per group
int halo_bn(int N) {
  return N <= 48 ? 48 : (N <= 64 ? 64 : (N <= 96 ? 96 : 128));
}

hipError_t run_halo(const HaloGeom& g, const uint16_t* src, const DenseK& lb,
                    const Epi& e, int K, int N, int groups, hipStream_t s) {
  const int bn = halo_bn(N);
  if (bn == 48)
    return launch_halo<64, false, 2>(g, src, lb, e, K, N, groups, s);
  if (bn == 64)
    return launch_halo<64, false, 0>(g, src, lb, e, K, N, groups, s);
  if (bn == 96)
    return launch_halo<96, false, 0>(g, src, lb, e, K, N, groups, s);
  return launch_halo<128, true, 0>(g, src, lb, e, K, N, groups, s);
}

}  // namespace

// conv forward, stride 1 (the s2d conv1 and AlexNet conv2..5 / VGG shapes):
// -2 when the halo path does not apply (the caller falls back to
// hvk_conv_fwd)
static int conv_fwd_halo(const void* X, const void* Wt, const float* bias,
                         void* Y, int N, int H, int W, int C, int OC, int KH,
                         int KW, int pt, int pl, int OH, int OW, int groups,
                         int act, const Q8* q8, hipStream_t s) {
  const int Cg = C / groups, OCg = OC / groups;
  HaloGeom g = make_halo(N, H, W, C, Cg, OH, OW, KH, KW, -pt, -pl, 0);
  const int K = KH * KW * Cg;
  // measured (profiles/r3_experiments.md §9): faster than the implicit GEMM
  // for the short reduction of AlexNet conv1 after space-to-depth (K = 432,
  // +16 %), slower for conv2 (K = 1200, -4 %)
  if (!halo_ok(g, halo_bn(OCg), X, Wt) || OCg % 8 || K > 1024) return -2;
  DenseK lb{(const uint16_t*)Wt, (long long)OCg * K, OCg, K, K, 1};
  Epi e = make_epi(Y, OC, N * OH * OW, OCg, 0, 0, 1.f, 0.f, bias, 1, act,
                   nullptr, 0, 0);
  e.gcol = OCg;
  if (q8) {
    if (!e.fast_ok() || OCg % 8 || (((uintptr_t)q8->q) & 7)) return -3;
    e.q8 = *q8;
  }
  return (int)run_halo(g, (const uint16_t*)X, lb, e, K, OCg, groups, s);
}

HVK_API int hvk_conv_fwd_halo(const void* X, const void* Wt, const float* bias,
                              void* Y, int N, int H, int W, int C, int OC,
                              int KH, int KW, int pt, int pl, int OH, int OW,
                              int groups, int act, hipStream_t s) {
  return conv_fwd_halo(X, Wt, bias, Y, N, H, W, C, OC, KH, KW, pt, pl, OH,
                       OW, groups, act, nullptr, s);
}

// as hvk_conv_fwd_halo, and the fp8 copy of Y for the fp8 layer reading it
// (q8: [N][OH][OW][OC] bytes; fmt 0 e4m3 / 1 e5m2; amax into the shards)
HVK_API int hvk_conv_fwd_halo_q8(const void* X, const void* Wt,
                                 const float* bias, void* Y, int N, int H,
                                 int W, int C, int OC, int KH, int KW, int pt,
                                 int pl, int OH, int OW, int groups, int act,
                                 void* q8, const float* q8_st, float* q8_shard,
                                 float q8_fmax, int q8_fmt, int hist,
                                 hipStream_t s) {
  const Q8 z{(uint8_t*)q8, q8_st, q8_shard, q8_fmax, q8_fmt, hist};
  return conv_fwd_halo(X, Wt, bias, Y, N, H, W, C, OC, KH, KW, pt, pl, OH,
                       OW, groups, act, &z, s);
}

// conv backward-data, stride 1, weights pre-permuted to Wt[g][c][kh][kw][oc]
// (as hvk_conv_dgrad_t): dX = conv(dY, flipped W); -2 when not applicable
HVK_API int hvk_conv_dgrad_halo(const void* dY, const void* Wt, void* dX,
                                int N, int H, int W, int C, int OC, int KH,
                                int KW, int pt, int pl, int OH, int OW,
                                int groups, const void* aux, int aux_act,
                                hipStream_t s) {
  const int Cg = C / groups, OCg = OC / groups;
  // dX pixel (h, w) reads dY (h + pt - kh, w + pl - kw): halo origin
  // (h0 + pt - KH + 1, w0 + pl - KW + 1), taps flipped
  HaloGeom g = make_halo(N, OH, OW, OC, OCg, H, W, KH, KW, pt - KH + 1,
                         pl - KW + 1, 1);
  const int K = KH * KW * OCg;
  if (!halo_ok(g, halo_bn(Cg), dY, Wt) || Cg % 8) return -2;
  DenseK lb{(const uint16_t*)Wt, (long long)K * Cg, Cg, K, K, 1};
  Epi e = make_epi(dX, C, N * H * W, Cg, 0, 0, 1.f, 0.f, nullptr, 0, 0, aux, C,
                   aux_act);
  e.gcol = Cg;
  return (int)run_halo(g, (const uint16_t*)dY, lb, e, K, Cg, groups, s);
}
