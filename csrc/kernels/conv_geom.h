// conv_geom.h - NHWC convolution geometry shared by the bf16 (gemm.hip) and
// fp8 (gemm_fp8.hip) implicit-GEMM kernels.  All index math in the loaders
// goes through FastDiv (one mul_hi + add + shift per division).
#pragma once
#include "hvk_common.h"

namespace hvk {

struct ConvGeom {
  int N, H, W, C, Cg;       // input NHWC, C total, Cg per group
  int OH, OW, OC, OCg;      // output
  int KH, KW, sy, sx, pt, pl;
  FastDiv fOW, fOHOW, fW, fHW, fCg, fOCg, fKW, fSy, fSx;
};

inline ConvGeom make_geom(int N, int H, int W, int C, int OC, int KH, int KW,
                          int sy, int sx, int pt, int pl, int OH, int OW,
                          int groups) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Cg = C / groups;
  g.OH = OH; g.OW = OW; g.OC = OC; g.OCg = OC / groups;
  g.KH = KH; g.KW = KW; g.sy = sy; g.sx = sx; g.pt = pt; g.pl = pl;
  g.fOW = make_fastdiv(OW); g.fOHOW = make_fastdiv(OH * OW);
  g.fW = make_fastdiv(W); g.fHW = make_fastdiv(H * W);
  g.fCg = make_fastdiv(g.Cg); g.fOCg = make_fastdiv(g.OCg);
  g.fKW = make_fastdiv(KW);
  g.fSy = make_fastdiv(sy);
  g.fSx = make_fastdiv(sx);
  return g;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ---------------------------------------------------------------------------
// Branch-free LDS-DMA addressing for the implicit-GEMM A operands ("fast"
// loaders, kFast in gemm.hip / gemm_fp8.hip): a tile row's pixel offset and
// two bit masks of the kh / kw taps that stay inside the image are computed
// once per block (DRow); a lane's 16-B chunk has the same k in every DMA slot,
// so its tap (kh, kw, channel) is decoded once per K tile (DTap) and shared.
// Per slot and tile the address is one add, two mask tests and a select.  The
// per-slot divisions and divergent bounds branches this replaces cost conv
// dgrad 30-38 % and conv forward 6-16 % of its rate on MI355X
// (profiles/gemm_experiments_r2.md §3).
struct DRow { int pix; uint32_t rm, cm; };
struct DTap { int off; uint32_t kh, kw, ok; };

// bits [lo, hi) of a 32-bit mask (clamped to [0, 32))
__device__ __forceinline__ uint32_t span_mask(int lo, int hi) {
  lo = max(lo, 0);
  hi = min(hi, 32);
  if (hi <= lo) return 0u;
  const uint32_t up = hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u);
  return up & ~((1u << lo) - 1u);
}

// p if bit 0 of v is set, else zp.  The empty asm pins the address
// computation before the select: without it hipcc sinks the 64-bit address
// math into an exec-mask branch around every DMA slot.
template <class T>
__device__ __forceinline__ const T* pick_ptr(const T* p, uint32_t v,
                                             const T* zp) {
  asm("" : "+v"(p));
  return (v & 1u) ? p : zp;
}

// conv forward, row m = output pixel (n, oh, ow): element offset x + pix +
// off; kh valid iff 0 <= oh*sy - pt + kh < H (bits of rm), kw likewise
__device__ __forceinline__ DRow fwd_drow(const ConvGeom& g, int M, int coff,
                                         int m) {
  DRow r;
  uint32_t mm = m < M ? m : 0, n, rem, oh, ow;
  fdivmod(mm, g.fOHOW, n, rem);
  fdivmod(rem, g.fOW, oh, ow);
  const int ih0 = (int)oh * g.sy - g.pt, iw0 = (int)ow * g.sx - g.pl;
  r.pix = (int)n * g.H * g.W * g.C + coff + (ih0 * g.W + iw0) * g.C;
  r.rm = m < M ? span_mask(-ih0, g.H - ih0) : 0u;
  r.cm = span_mask(-iw0, g.W - iw0);
  return r;
}
__device__ __forceinline__ DTap fwd_dtap(const ConvGeom& g, int K, int k) {
  DTap t;
  t.ok = k < K ? 1u : 0u;
  uint32_t tp, ch, kh, kw;
  fdivmod(t.ok ? k : 0, g.fCg, tp, ch);
  fdivmod(tp, g.fKW, kh, kw);
  t.kh = kh;
  t.kw = kw;
  t.off = ((int)kh * g.W + (int)kw) * g.C + (int)ch;
  return t;
}
// conv dgrad (stride 1), row m = input pixel (n, h, w): dY offset dy + pix +
// off with oh = h + pt - kh, ow = w + pl - kw
__device__ __forceinline__ DRow dgrad_drow(const ConvGeom& g, int M, int coff,
                                           int m) {
  DRow r;
  uint32_t mm = m < M ? m : 0, n, rem, h, w;
  fdivmod(mm, g.fHW, n, rem);
  fdivmod(rem, g.fW, h, w);
  const int hp = (int)h + g.pt, wp = (int)w + g.pl;
  r.pix = (int)n * g.OH * g.OW * g.OC + coff + (hp * g.OW + wp) * g.OC;
  r.rm = m < M ? span_mask(hp - g.OH + 1, hp + 1) : 0u;
  r.cm = span_mask(wp - g.OW + 1, wp + 1);
  return r;
}
__device__ __forceinline__ DTap dgrad_dtap(const ConvGeom& g, int K, int k) {
  DTap t;
  t.ok = k < K ? 1u : 0u;
  uint32_t tp, oc, kh, kw;
  fdivmod(t.ok ? k : 0, g.fOCg, tp, oc);
  fdivmod(tp, g.fKW, kh, kw);
  t.kh = kh;
  t.kw = kw;
  t.off = (int)oc - ((int)kh * g.OW + (int)kw) * g.OC;
  return t;
}
__device__ __forceinline__ uint32_t tap_ok(const DRow& r, const DTap& t) {
  return t.ok & (r.rm >> t.kh) & (r.cm >> t.kw);
}

// LDS-DMA through a buffer descriptor (buffer_load_dwordx4 ... lds): 32-bit
// byte offsets instead of 64-bit addresses, and the hardware bounds check
// replaces the zero page - a lane whose offset is kBufOOB reads zeros
// (verified on gfx950: tools/probes/buffer_lds_oob.hip).  Tensors must span
// less than 2 GiB from the descriptor base (loaders' buf_ok()).
constexpr uint32_t kBufOOB = 0x80000000u;
constexpr long long kBufMaxBytes = (1ll << 31) - 64;
// The base is read through readfirstlane so that hipcc can PROVE the
// descriptor wave-uniform; otherwise it wraps every buffer op in a waterfall
// loop (cdna_hip_programming.md T20 - seen here on the 128-wide conv kernel).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(const void* base) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  void* p = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)kBufOOB,
                                           0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds,
                                      uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
// byte offset of element `off` if bit 0 of v is set, else kBufOOB
__device__ __forceinline__ uint32_t buf_off(int off, uint32_t v) {
  return (v & 1u) ? (uint32_t)off * 2u : kBufOOB;
}

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md T1):
// consecutive logical workgroup ids land on one XCD (private L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace hvk
