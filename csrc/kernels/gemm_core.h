// gemm_core.h - MFMA (v_mfma_f32_16x16x32_bf16) GEMM and implicit-GEMM
// convolution for gfx950: loaders, epilogue, main loop and launch policy.
// The entry points are split over gemm.hip (dense), gemm_conv_fwd.hip,
// gemm_conv_dgrad.hip and gemm_conv_wgrad.hip so that they compile in
// parallel.
//
// One main loop, pluggable operand loaders and epilogues:
//   * C[M][N] = alpha * op(A) * op(B) (+ beta*C) (+ bias) -> act -> store
//   * conv forward   : A = im2col(X) gathered on the fly (NHWC), B = W
//   * conv dgrad     : A = "transposed im2col" of dY, B = W rows gathered
//   * conv wgrad     : A = dY^T, B = im2col(X), split over pixels, f32 atomics
// Replaces the reference's ocl/gemm.cl + matrix_multiplication*.cl family and
// the (absent) Znicz conv/all2all/gd kernels.
//
// Block tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 =
// 4x4 MFMA 16x16 tiles - or, for most LDS-DMA shapes, 512 threads = 8 waves
// (2x4, each 64x32) on the same tile and LDS footprint (see want_w8).  Operands are register-staged global->LDS (async
// STAGE split: next tile's global loads are issued before this tile's MFMAs,
// written to the other LDS buffer after them), double buffered, one barrier
// per K-tile.  LDS images:
//   K-major  tile [128 rows][64 k]  128-B rows, 16-B chunk c stored at
//            c ^ (row & 7)   -> ds_read_b128 fragment reads conflict-free
//   MN-major tile [64 k][128 cols]  256-B rows, 32-B block b stored at
//            b ^ h(k), h(k) = (k&3) | ((k>>3)&1)<<2 -> ds_read_b64_tr_b16
//            transposed fragment reads conflict-free
// Grid x is remapped so that consecutive output tiles share one XCD's L2.
#pragma once
#include <type_traits>

#include "conv_geom.h"
#include "fp8_common.h"

using namespace hvk;

// GEMM schedule selector, one per library (defined in gemm.hip)
extern int hvk_gemm_variant;

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int TILE = 128 * 64;  // elements per operand tile buffer

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }

// Source pages for LDS-DMA loads: out-of-bounds lanes read zeros, the fused
// bias-gradient column reads (1, 0, ..., 0).
__device__ __attribute__((aligned(16))) const uint16_t g_zero8[8] = {0};
__device__ __attribute__((aligned(16))) const uint16_t g_ones8[8] = {
    0x3F80, 0, 0, 0, 0, 0, 0, 0};

__device__ __forceinline__ uint4 pack8(const uint16_t* e) {
  uint4 v;
  v.x = e[0] | ((uint32_t)e[1] << 16);
  v.y = e[2] | ((uint32_t)e[3] << 16);
  v.z = e[4] | ((uint32_t)e[5] << 16);
  v.w = e[6] | ((uint32_t)e[7] << 16);
  return v;
}

// ---------------------------------------------------------------- loaders
// DMA source: p if bit 0 of v is set, else zp (the zero page by default)
// - see hvk::pick_ptr in conv_geom.h.
__device__ __forceinline__ const uint16_t* pick_src(
    const uint16_t* p, uint32_t v, const uint16_t* zp = g_zero8) {
  return pick_ptr(p, v, zp);
}

// the per-slot state type of a fast MN-major B loader (int placeholder else)
template <class L, bool F> struct DColOf { using type = int; };
template <class L> struct DColOf<L, true> { using type = typename L::DCol; };

// K-major loader: rows = M (or N) index, 8-element chunks along K.
struct DenseK {
  const uint16_t* p;
  long long gstride;  // elements between groups
  int rows, K, ld, vec;
  struct Ctx { const uint16_t* row; int ok; };
  __device__ void group(int g) { p += (long long)g * gstride; }
  __device__ __forceinline__ Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < rows;
    c.row = p + (long long)(c.ok ? r : 0) * ld;
    return c;
  }
  static constexpr bool kGlds = true;
  static constexpr bool kFast = false;
  static constexpr bool kBuf = true;
  __host__ __device__ bool dma_ok() const { return vec && (K & 7) == 0; }
  __device__ __forceinline__ const uint16_t* src(const Ctx& c, int k) const {
    // bitwise condition: && made hipcc branch around the address
    return pick_src(c.row + k, (c.ok != 0) & (k < K));
  }
  // buffer DMA: descriptor at the (group) base, per-slot row byte offset
  bool buf_ok(int groups) const {
    return ((long long)(rows - 1) * ld + K) * 2 +
               (long long)(groups - 1) * gstride * 2 < kBufMaxBytes;
  }
  __device__ const void* dbase() const { return p; }
  __device__ __forceinline__ uint32_t row_voff(int r) const {
    return r < rows ? (uint32_t)r * (uint32_t)ld * 2u : kBufOOB;
  }
  __device__ __forceinline__ uint4 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero4();
    if (vec && k + 8 <= K) return *(const uint4*)(c.row + k);
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = (k + j < K) ? c.row[k + j] : 0;
    return pack8(e);
  }
};

// MN-major loader: rows = K index, 8-element chunks along M (or N).
struct DenseMN {
  const uint16_t* p;
  long long gstride;
  int cols, K, ld, vec;
  int ones_col;  // >= 0: column of ones appended at index cols (bias grad)
  struct Ctx { int c; };
  __device__ void group(int g) { p += (long long)g * gstride; }
  __device__ __forceinline__ Ctx col_ctx(int c) const { return Ctx{c}; }
  static constexpr bool kGlds = true;
  static constexpr bool kFast = false;
  // buffer DMA only without the ones column (its page is another tensor)
  static constexpr bool kBuf = true;
  bool buf_ok(int groups) const {
    return ones_col < 0 &&
           ((long long)(K - 1) * ld + cols) * 2 +
                   (long long)(groups - 1) * gstride * 2 < kBufMaxBytes;
  }
  __device__ const void* dbase() const { return p; }
  // byte offset of chunk column c in k-row kr (kBufOOB past the columns)
  __device__ __forceinline__ uint32_t col_voff(int c, int kr) const {
    return c < cols ? ((uint32_t)kr * (uint32_t)ld + (uint32_t)c) * 2u
                    : kBufOOB;
  }
  __host__ __device__ bool dma_ok() const {
    return vec && (cols & 7) == 0 && (ones_col < 0 || (ones_col & 7) == 0);
  }
  __device__ __forceinline__ const uint16_t* src(const Ctx& cx, int k) const {
    // branch-free: in range -> data, the ones column -> ones page, else zeros
    const bool in = k < K;
    const uint16_t* zp = (in & (cx.c == ones_col)) ? g_ones8 : g_zero8;
    return pick_src(p + (long long)k * ld + cx.c, in & (cx.c < cols), zp);
  }
  __device__ __forceinline__ uint4 load(const Ctx& cx, int k) const {
    if (k >= K) return zero4();
    const uint16_t* row = p + (long long)k * ld;
    if (vec && cx.c + 8 <= cols) return *(const uint4*)(row + cx.c);
    if (cx.c >= cols && (ones_col < 0 || cx.c > ones_col)) return zero4();
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int c = cx.c + j;
      e[j] = c < cols ? row[c] : (c == ones_col ? (uint16_t)0x3F80 : 0);
    }
    return pack8(e);
  }
};


// conv forward A: rows = output pixels (n,oh,ow), k = (kh,kw,c)
struct ConvFwdA {
  const uint16_t* x;
  ConvGeom g;
  int M, K, vec;
  int coff;
  struct Ctx { int base, ih0, iw0, ok; };
  __device__ void group(int gi) { coff = gi * g.Cg; }
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < M;
    uint32_t mm = c.ok ? m : 0, n, rem, oh, ow;
    fdivmod(mm, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    c.base = n * g.H * g.W * g.C + coff;
    c.ih0 = oh * g.sy - g.pt;
    c.iw0 = ow * g.sx - g.pl;
    return c;
  }
  __device__ __forceinline__ uint16_t elem(const Ctx& c, int k) const {
    if (k >= K) return 0;
    uint32_t t, ch, kh, kw;
    fdivmod(k, g.fCg, t, ch);
    fdivmod(t, g.fKW, kh, kw);
    int ih = c.ih0 + (int)kh, iw = c.iw0 + (int)kw;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return 0;
    return x[c.base + (ih * g.W + iw) * g.C + ch];
  }
  static constexpr bool kGlds = true;
  static constexpr bool kFast = true;
  __host__ __device__ bool dma_ok() const { return vec && g.KH <= 32 && g.KW <= 32; }
  __device__ __forceinline__ const uint16_t* src(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return g_zero8;
    uint32_t t, ch, kh, kw;
    fdivmod(k, g.fCg, t, ch);
    fdivmod(t, g.fKW, kh, kw);
    int ih = c.ih0 + (int)kh, iw = c.iw0 + (int)kw;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
      return g_zero8;
    return x + c.base + (ih * g.W + iw) * g.C + ch;
  }
  // fast DMA addressing (conv_geom.h): x + pix + off, kh in rm, kw in cm
  __device__ __forceinline__ DRow drow(int m) const {
    return fwd_drow(g, M, coff, m);
  }
  __device__ __forceinline__ DTap dtap(int k) const { return fwd_dtap(g, K, k); }
  __device__ __forceinline__ const uint16_t* dsrc(const DRow& r,
                                                  const DTap& t) const {
    return pick_src(x + (r.pix + t.off), tap_ok(r, t));
  }
  static constexpr bool kBuf = true;
  bool buf_ok(int) const {
    return (long long)g.N * g.H * g.W * g.C * 2 < kBufMaxBytes;
  }
  __device__ const void* dbase() const { return x; }
  __device__ __forceinline__ uint32_t dvoff(const DRow& r,
                                            const DTap& t) const {
    return buf_off(r.pix + t.off, tap_ok(r, t));
  }
  __device__ __forceinline__ uint4 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero4();
    if (vec) {  // Cg % 8 == 0: the 8 elements are 8 channels of one tap
      uint32_t t, ch, kh, kw;
      fdivmod(k, g.fCg, t, ch);
      fdivmod(t, g.fKW, kh, kw);
      int ih = c.ih0 + (int)kh, iw = c.iw0 + (int)kw;
      if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
        return zero4();
      return *(const uint4*)(x + c.base + (ih * g.W + iw) * g.C + ch);
    }
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = elem(c, k + j);
    return pack8(e);
  }
};

// conv dgrad A: rows = input pixels (n,h,w), k = (kh,kw,oc) over dY
struct ConvDgradA {
  const uint16_t* dy;
  ConvGeom g;
  int M, K, vec;
  int coff;
  struct Ctx { int base, hp, wp, ok; };
  __device__ void group(int gi) { coff = gi * g.OCg; }
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < M;
    uint32_t mm = c.ok ? m : 0, n, rem, h, w;
    fdivmod(mm, g.fHW, n, rem);
    fdivmod(rem, g.fW, h, w);
    c.base = n * g.OH * g.OW * g.OC + coff;
    c.hp = h + g.pt;
    c.wp = w + g.pl;
    return c;
  }
  __device__ __forceinline__ int tap(const Ctx& c, int k, uint32_t& oc) const {
    uint32_t t, kh, kw;
    fdivmod(k, g.fOCg, t, oc);
    fdivmod(t, g.fKW, kh, kw);
    int ohs = c.hp - (int)kh, ows = c.wp - (int)kw;
    if (ohs < 0 || ows < 0) return -1;
    if (g.sy == 1 && g.sx == 1) {  // stride 1: no divisions (uniform branch)
      if (ohs >= g.OH || ows >= g.OW) return -1;
      return c.base + (ohs * g.OW + ows) * g.OC;
    }
    int oh = (int)fdiv((uint32_t)ohs, g.fSy), ow = (int)fdiv((uint32_t)ows, g.fSx);
    if (oh * g.sy != ohs || ow * g.sx != ows || oh >= g.OH || ow >= g.OW)
      return -1;
    return c.base + (oh * g.OW + ow) * g.OC;
  }
  static constexpr bool kGlds = true;
  // stride 1 only (strided dgrad: ConvDgradAStr)
  static constexpr bool kFast = true;
  __host__ __device__ bool dma_ok() const {
    return vec && g.sy == 1 && g.sx == 1 && g.KH <= 32 && g.KW <= 32;
  }
  __device__ __forceinline__ const uint16_t* src(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return g_zero8;
    uint32_t oc;
    int off = tap(c, k, oc);
    return off < 0 ? g_zero8 : dy + off + oc;
  }
  // fast DMA addressing (stride 1, conv_geom.h): oh = hp - kh, ow = wp - kw
  __device__ __forceinline__ DRow drow(int m) const {
    return dgrad_drow(g, M, coff, m);
  }
  __device__ __forceinline__ DTap dtap(int k) const {
    return dgrad_dtap(g, K, k);
  }
  __device__ __forceinline__ const uint16_t* dsrc(const DRow& r,
                                                  const DTap& t) const {
    return pick_src(dy + (r.pix + t.off), tap_ok(r, t));
  }
  static constexpr bool kBuf = true;
  bool buf_ok(int) const {
    return (long long)g.N * g.OH * g.OW * g.OC * 2 < kBufMaxBytes;
  }
  __device__ const void* dbase() const { return dy; }
  __device__ __forceinline__ uint32_t dvoff(const DRow& r,
                                            const DTap& t) const {
    return buf_off(r.pix + t.off, tap_ok(r, t));
  }
  __device__ __forceinline__ uint4 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero4();
    if (vec) {
      uint32_t oc;
      int off = tap(c, k, oc);
      if (off < 0) return zero4();
      return *(const uint4*)(dy + off + oc);
    }
    return zero4();  // OC % 8 != 0 uses ConvDgradAS
  }
};

// strided dgrad: per-slot src() addressing (the tap must divide by stride)
struct ConvDgradAStr : ConvDgradA {
  static constexpr bool kFast = false;
  static constexpr bool kBuf = false;
  bool buf_ok(int) const { return false; }
  __host__ __device__ bool dma_ok() const { return vec; }
};

// scalar-gather variant for OC % 8 != 0 (a separate instantiation: its
// 8-tap loop pushes the loader struct into scratch, which must not happen
// to the common vectorised kernels)
struct ConvDgradAS : ConvDgradA {
  static constexpr bool kGlds = false;
  static constexpr bool kFast = false;
  static constexpr bool kBuf = false;
  bool buf_ok(int) const { return false; }
  __host__ __device__ bool dma_ok() const { return false; }
  __device__ uint4 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero4();
    uint16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      e[j] = 0;
      if (k + j < K) {
        uint32_t oc;
        int off = tap(c, k + j, oc);
        if (off >= 0) e[j] = dy[off + oc];
      }
    }
    return pack8(e);
  }
};

// conv wgrad B: MN-major, rows = output pixel p, cols kk = (kh,kw,c)
struct ConvWgradB {
  const uint16_t* x;
  ConvGeom g;
  int K /* pixels */, KK, vec;
  int coff;
  int ones;  // append a ones column at index KK (bias gradient)
  struct Ctx { int kh, kw, ch, ok; };
  __device__ void group(int gi) { coff = gi * g.Cg; }
  __device__ __forceinline__ Ctx col_ctx(int kk) const {
    Ctx c;
    c.ok = kk < KK ? 1 : ((ones && kk == KK) ? 2 : 0);
    uint32_t t, ch, kh, kw;
    fdivmod(c.ok ? kk : 0, g.fCg, t, ch);
    fdivmod(t, g.fKW, kh, kw);
    c.kh = kh; c.kw = kw; c.ch = ch;
    return c;
  }
  static constexpr bool kGlds = true;
  // fast DMA addressing needs OH*OW >= BK (a running pixel position wraps
  // into the next image at most once per K tile); else ConvWgradBGen
  static constexpr bool kFast = true;
  static constexpr bool kBuf = false;
  bool buf_ok(int) const { return false; }
  __host__ __device__ bool dma_ok() const { return vec && (KK & 7) == 0; }
  // per DMA slot: the column's tap (fixed) and a running pixel p with
  // rem = p mod OH*OW and the image base, advanced by BK per tile - one
  // division per slot and tile (rem -> oh, ow) instead of two, no branches
  struct DCol { int ch, kh, kw; uint32_t kind; int p, rem, nbase; };
  __device__ __forceinline__ DCol dcol(int kk, int p, bool zero) const {
    DCol d;
    d.kind = zero ? 0u : kk < KK ? 1u : ((ones && kk == KK) ? 2u : 0u);
    uint32_t t, ch, kh, kw, n, rem;
    fdivmod(d.kind == 1u ? kk : 0, g.fCg, t, ch);
    fdivmod(t, g.fKW, kh, kw);
    d.ch = coff + (int)ch;
    d.kh = (int)kh - g.pt;
    d.kw = (int)kw - g.pl;
    d.p = p;
    fdivmod((uint32_t)p, g.fOHOW, n, rem);
    d.rem = (int)rem;
    d.nbase = (int)n * g.H * g.W * g.C;
    return d;
  }
  __device__ __forceinline__ const uint16_t* dsrc(const DCol& d) const {
    uint32_t oh, ow;
    fdivmod((uint32_t)d.rem, g.fOW, oh, ow);
    const int ih = (int)oh * g.sy + d.kh, iw = (int)ow * g.sx + d.kw;
    const uint32_t in = (d.p < K ? 1u : 0u);
    const uint32_t v = in & (d.kind == 1u ? 1u : 0u) &
                       ((unsigned)ih < (unsigned)g.H ? 1u : 0u) &
                       ((unsigned)iw < (unsigned)g.W ? 1u : 0u);
    const uint16_t* zp =
        (in & (d.kind == 2u ? 1u : 0u)) ? g_ones8 : g_zero8;
    return pick_src(x + (d.nbase + (ih * g.W + iw) * g.C + d.ch), v, zp);
  }
  __device__ __forceinline__ void dnext_by(DCol& d, int step) const {
    d.p += step;
    d.rem += step;
    const bool w = d.rem >= g.OH * g.OW;
    d.rem -= w ? g.OH * g.OW : 0;
    d.nbase += w ? g.H * g.W * g.C : 0;
  }
  __device__ __forceinline__ void dnext(DCol& d) const { dnext_by(d, BK); }
  __device__ __forceinline__ const uint16_t* src(const Ctx& cx, int p) const {
    if (!cx.ok || p >= K) return g_zero8;
    if (cx.ok == 2) return g_ones8;
    uint32_t n, rem, oh, ow;
    fdivmod(p, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    int ih = oh * g.sy - g.pt + cx.kh, iw = ow * g.sx - g.pl + cx.kw;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
      return g_zero8;
    return x + (long long)n * g.H * g.W * g.C + coff + (ih * g.W + iw) * g.C +
           cx.ch;
  }
  __device__ __forceinline__ uint4 load(const Ctx& cx, int p) const {
    if (!cx.ok || p >= K) return zero4();
    if (cx.ok == 2) return make_uint4(0x3F80u, 0, 0, 0);
    uint32_t n, rem, oh, ow;
    fdivmod(p, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    int ih0 = oh * g.sy - g.pt, iw0 = ow * g.sx - g.pl;
    long long base = (long long)n * g.H * g.W * g.C + coff;
    if (vec) {
      int ih = ih0 + cx.kh, iw = iw0 + cx.kw;
      if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
        return zero4();
      return *(const uint4*)(x + base + (ih * g.W + iw) * g.C + cx.ch);
    }
    uint16_t e[8];
    uint32_t kk0 = 0;
    (void)kk0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // element j is column kk+j: recompute its tap
      int kk = (cx.kh * g.KW + cx.kw) * g.Cg + cx.ch + j;
      e[j] = 0;
      if (ones && kk == KK) e[j] = 0x3F80;
      if (kk < KK) {
        uint32_t t, ch, kh, kw;
        fdivmod(kk, g.fCg, t, ch);
        fdivmod(t, g.fKW, kh, kw);
        int ih = ih0 + (int)kh, iw = iw0 + (int)kw;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          e[j] = x[base + (ih * g.W + iw) * g.C + ch];
      }
    }
    return pack8(e);
  }
};


// wgrad B for OH * OW < BK: per-slot src() addressing
struct ConvWgradBGen : ConvWgradB {
  static constexpr bool kFast = false;
};

// Small-channel convs (C % 8 != 0, groups == 1, e.g. AlexNet conv1 with
// C = 3): K is re-laid out as (kh, j) with j < RUNP, where j < RUN = KW*C
// indexes the CONTIGUOUS (kw, c) run of one input row and RUNP pads it to
// a multiple of 8 (weights zero there).  A chunk of 8 k's is then 8
// consecutive input elements: one (2-byte aligned) 16-B load; gfx950 runs
// in unaligned-access mode, hipcc emits global_load_dwordx4 for it.
__device__ __forceinline__ uint4 ld16u(const uint16_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}

struct RunGeom {
  int RUN, RUNP;
  FastDiv fRUNP, fC;
  long long total;  // elements of x (tail guard)
};

struct ConvFwdRunA {
  static constexpr bool kGlds = false;
  static constexpr bool kFast = false;
  static constexpr bool kBuf = false;
  bool buf_ok(int) const { return false; }
  __host__ __device__ bool dma_ok() const { return false; }
  const uint16_t* x;
  ConvGeom g;
  RunGeom r;
  int M, K;  // K = KH * RUNP
  struct Ctx { long long base; int ih0, iw0, ok, full; };
  __device__ void group(int) {}
  __device__ __forceinline__ Ctx row_ctx(int m) const {
    Ctx c;
    c.ok = m < M;
    uint32_t mm = c.ok ? m : 0, n, rem, oh, ow;
    fdivmod(mm, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    c.base = (long long)n * g.H * g.W * g.C;
    c.ih0 = oh * g.sy - g.pt;
    c.iw0 = ow * g.sx - g.pl;
    c.full = c.iw0 >= 0 && c.iw0 + g.KW <= g.W;
    return c;
  }
  __device__ __forceinline__ uint4 load(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return zero4();
    uint32_t kh, j;
    fdivmod(k, r.fRUNP, kh, j);
    int ih = c.ih0 + (int)kh;
    if ((unsigned)ih >= (unsigned)g.H) return zero4();
    long long a = c.base + ((long long)ih * g.W + c.iw0) * g.C + j;
    if (c.full && a + 8 <= r.total) return ld16u(x + a);
    uint16_t e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int jj = (int)j + q;
      e[q] = 0;
      if (jj < r.RUN) {
        uint32_t kw, ch;
        fdivmod(jj, r.fC, kw, ch);
        int iw = c.iw0 + (int)kw;
        if ((unsigned)iw < (unsigned)g.W)
          e[q] = x[c.base + ((long long)ih * g.W + iw) * g.C + ch];
      }
    }
    return pack8(e);
  }
};

// wgrad B for small-channel convs: MN-major, rows = pixels, cols = (kh, j)
struct ConvWgradRunB {
  static constexpr bool kGlds = false;
  static constexpr bool kFast = false;
  static constexpr bool kBuf = false;
  bool buf_ok(int) const { return false; }
  __host__ __device__ bool dma_ok() const { return false; }
  const uint16_t* x;
  ConvGeom g;
  RunGeom r;
  int K /* pixels */, KK /* KH*RUNP */, ones;
  struct Ctx { int kh, j, ok; };
  __device__ void group(int) {}
  __device__ __forceinline__ Ctx col_ctx(int kk) const {
    Ctx c;
    c.ok = kk < KK ? 1 : ((ones && kk == KK) ? 2 : 0);
    uint32_t kh, j;
    fdivmod(kk < KK ? kk : 0, r.fRUNP, kh, j);
    c.kh = kh;
    c.j = j;
    return c;
  }
  __device__ __forceinline__ uint4 load(const Ctx& cx, int p) const {
    if (!cx.ok || p >= K) return zero4();
    if (cx.ok == 2) return make_uint4(0x3F80u, 0, 0, 0);
    uint32_t n, rem, oh, ow;
    fdivmod(p, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    int ih = oh * g.sy - g.pt + cx.kh;
    if ((unsigned)ih >= (unsigned)g.H) return zero4();
    int iw0 = ow * g.sx - g.pl;
    long long base = (long long)n * g.H * g.W * g.C;
    long long a = base + ((long long)ih * g.W + iw0) * g.C + cx.j;
    if (iw0 >= 0 && iw0 + g.KW <= g.W && a + 8 <= r.total) {
      uint4 v = ld16u(x + a);
      if (cx.j + 8 > r.RUN) {  // zero the pad tail of the run
        uint16_t* h = (uint16_t*)&v;
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (cx.j + q >= r.RUN) h[q] = 0;
      }
      return v;
    }
    uint16_t e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int jj = cx.j + q;
      e[q] = 0;
      if (jj < r.RUN) {
        uint32_t kw, ch;
        fdivmod(jj, r.fC, kw, ch);
        int iw = iw0 + (int)kw;
        if ((unsigned)iw < (unsigned)g.W)
          e[q] = x[base + ((long long)ih * g.W + iw) * g.C + ch];
      }
    }
    return pack8(e);
  }
};

// -------------------------------------------------------------- epilogue
struct Epi {
  void* c;
  int ldc, M, N;
  int out_f32;     // 1: float output, 0: bf16
  int atomic;      // 1: f32 atomicAdd (split-K / accumulate)
  float alpha, beta;
  const float* bias;
  int bias_mode;   // 0 none, 1 per column, 2 per row
  int act;         // forward activation after bias
  const uint16_t* aux;  // multiply by act_bwd(aux, aux_act)
  int ld_aux, aux_act;
  int grow, gcol;  // per-group row / column offsets
  float* preact;   // optional f32 copy of the pre-activation (unused = null)
  int ones_col;    // column routed to bias_grad[m] (fused bias gradient)
  float* bias_grad;
  int bias_store;  // 1: the bias-gradient column is stored, not added
  int run_in, run_out;  // column remap n = kh*run_in + j -> kh*run_out + j
  // 1: split-K partial sums, each K split stored (not added) to its own
  // slice of an f32 workspace [splits][M][ldc] (grow = M: the split index
  // takes the group index's place in the row offset); 128-row gemm_kernel
  // tiles only
  int slice;
  // fused fp8 copy of the (bf16) output for the fp8 layer reading it
  // (store8_fast only; q8.q == nullptr: off)
  Q8 q8;
  __device__ __forceinline__ void store(int gi, int m, int n, float v) const {
    if (m >= M || n >= N) return;
    if (n == ones_col) {
      if (bias_store) bias_grad[m + gi * grow] = v * alpha;
      else atomicAdd(bias_grad + m + gi * grow, v * alpha);
      return;
    }
    if (run_in) {
      int kh = n / run_in, j = n - kh * run_in;
      if (j >= run_out) return;
      n = kh * run_out + j;
    }
    int gm = m + gi * grow, gn = n + gi * gcol;
    long long idx = (long long)gm * ldc + gn;
    v *= alpha;
    if (bias_mode == 1) v += bias[gn];
    else if (bias_mode == 2) v += bias[gm];
    if (atomic) {
      atomicAdd((float*)c + idx, v);
      return;
    }
    if (beta != 0.f) {
      float old = out_f32 ? ((float*)c)[idx] : bf2f(((uint16_t*)c)[idx]);
      v += beta * old;
    }
    if (act) v = act_fwd(v, act);
    if (aux) v *= act_bwd(bf2f(aux[(long long)gm * ld_aux + gn]), aux_act);
    if (out_f32) ((float*)c)[idx] = v;
    else ((uint16_t*)c)[idx] = f2bf(v);
  }
  // The common case, decided once per block (wave-uniform): no atomics or
  // remaps, per-column bias, 16-B aligned rows.  Then every 8-column chunk
  // (except one holding the fused bias-gradient column) is one straight-line
  // store; beta != 0 adds beta * C (the gradient accumulation of an unsplit
  // weight-gradient GEMM: read-modify-write instead of f32 atomics).
  __host__ __device__ __forceinline__ bool fast_ok() const {
    return !atomic && !run_in && bias_mode != 2 && (ldc & 7) == 0 &&
           (((uintptr_t)c) & 15) == 0 &&
           (gcol & 7) == 0 &&
           (bias_mode != 1 || (((uintptr_t)bias) & 15) == 0) &&
           (!aux || ((ld_aux & 7) == 0 && (((uintptr_t)aux) & 15) == 0));
  }
  // fast_ok() and n + 8 <= N: one switch per chunk, vector bias / aux loads,
  // packed bf16 conversion (v is scratch)
  __device__ __forceinline__ void store8_fast(int gi, int m, int n,
                                              float* v, float qs = 1.f,
                                              float* amax = nullptr) const {
    const int gm = m + gi * grow, gn = n + gi * gcol;
    const long long idx = (long long)gm * ldc + gn;
    if (alpha != 1.f) {
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] *= alpha;
    }
    if (beta != 0.f) {
      float o[8];
      if (out_f32) {
        const float4* d = (const float4*)((const float*)c + idx);
        const float4 lo = d[0], hi = d[1];
        o[0] = lo.x; o[1] = lo.y; o[2] = lo.z; o[3] = lo.w;
        o[4] = hi.x; o[5] = hi.y; o[6] = hi.z; o[7] = hi.w;
      } else {
        const uint4 ov = *(const uint4*)((const uint16_t*)c + idx);
        const uint16_t* oh = (const uint16_t*)&ov;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = bf2f(oh[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += beta * o[q];
    }
    if (bias_mode == 1) {
      const float4 b0 = *(const float4*)(bias + gn);
      const float4 b1 = *(const float4*)(bias + gn + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    act_fwd8(v, act);
    if (aux) {
      const uint4 av = *(const uint4*)(aux + (long long)gm * ld_aux + gn);
      const uint16_t* ah = (const uint16_t*)&av;
      float a[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = bf2f(ah[q]);
      act_bwd_mul8(v, a, aux_act);
    }
    if (out_f32) {
      float4* d = (float4*)((float*)c + idx);
      d[0] = make_float4(v[0], v[1], v[2], v[3]);
      d[1] = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      const uint4 ob = pack_bf16x8(v);
      *(uint4*)((uint16_t*)c + idx) = ob;
      if (amax && q8.q) q8_store8(q8, idx, ob, qs, *amax);
    }
  }
  // 4 consecutive columns of one row from a lane's accumulator register
  // quad (the T4 loop's direct epilogue: no LDS staging); fast_ok(), no
  // fused fp8 copy, n % 4 == 0 and n + 4 <= N (v is scratch)
  __device__ __forceinline__ void store4_fast(int gi, int m, int n,
                                              float* v) const {
    const int gm = m + gi * grow, gn = n + gi * gcol;
    const long long idx = (long long)gm * ldc + gn;
    if (alpha != 1.f) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] *= alpha;
    }
    if (beta != 0.f) {
      float o[4];
      if (out_f32) {
        const float4 d = *(const float4*)((const float*)c + idx);
        o[0] = d.x; o[1] = d.y; o[2] = d.z; o[3] = d.w;
      } else {
        const uint2 ov = *(const uint2*)((const uint16_t*)c + idx);
        const uint16_t* oh = (const uint16_t*)&ov;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = bf2f(oh[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += beta * o[q];
    }
    if (bias_mode == 1) {
      const float4 b = *(const float4*)(bias + gn);
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    act_fwd_n<4>(v, act);
    if (aux) {
      const uint2 av = *(const uint2*)(aux + (long long)gm * ld_aux + gn);
      const uint16_t* ah = (const uint16_t*)&av;
      float a[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] = bf2f(ah[q]);
      act_bwd_mul_n<4>(v, a, aux_act);
    }
    if (out_f32) {
      *(float4*)((float*)c + idx) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      *(uint2*)((uint16_t*)c + idx) =
          make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
  // 4 consecutive columns of one row, finished in registers and packed to
  // bf16 (the T4 register epilogue): alpha, per-column bias, activation,
  // derivative of the layer below; fast_ok(), beta == 0, n % 4 == 0
  __device__ __forceinline__ uint2 pre4(int gi, int m, int n, float* v) const {
    const int gm = m + gi * grow, gn = n + gi * gcol;
    if (alpha != 1.f) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] *= alpha;
    }
    if (bias_mode == 1) {
      const float4 b = *(const float4*)(bias + gn);
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    act_fwd_n<4>(v, act);
    if (aux) {
      const uint2 av = *(const uint2*)(aux + (long long)gm * ld_aux + gn);
      float a[4];
      a[0] = __uint_as_float(av.x << 16);
      a[1] = __uint_as_float(av.x & 0xffff0000u);
      a[2] = __uint_as_float(av.y << 16);
      a[3] = __uint_as_float(av.y & 0xffff0000u);
      act_bwd_mul_n<4>(v, a, aux_act);
    }
    return make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
  // 8 consecutive columns of one row: 16-B vector stores when possible
  __device__ __forceinline__ void store8(int gi, int m, int n,
                                         const float* v) const {
    if (m >= M || n >= N) return;
    int gm = m + gi * grow, gn = n + gi * gcol;
    long long idx = (long long)gm * ldc + gn;
    const bool vecok = !atomic && !run_in && ones_col < 0 && n + 8 <= N &&
                       beta == 0.f && bias_mode != 2 && (ldc & 7) == 0 &&
                       (((uintptr_t)c) & 15) == 0 && (gn & 7) == 0 &&
                       (!aux || (ld_aux & 7) == 0);
    if (!vecok) {
#pragma unroll
      for (int q = 0; q < 8; ++q) store(gi, m, n + q, v[q]);
      return;
    }
    float o[8];
    float a[8];
    if (aux) {
      uint4 av = *(const uint4*)(aux + (long long)gm * ld_aux + gn);
      const uint16_t* ah = (const uint16_t*)&av;
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = act_bwd(bf2f(ah[q]), aux_act);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float t = v[q] * alpha;
      if (bias_mode == 1) t += bias[gn + q];
      if (act) t = act_fwd(t, act);
      if (aux) t *= a[q];
      o[q] = t;
    }
    if (out_f32) {
      float4* d = (float4*)((float*)c + idx);
      d[0] = make_float4(o[0], o[1], o[2], o[3]);
      d[1] = make_float4(o[4], o[5], o[6], o[7]);
    } else {
      uint4 w;
      w.x = f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
      w.y = f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
      w.z = f2bf(o[4]) | ((uint32_t)f2bf(o[5]) << 16);
      w.w = f2bf(o[6]) | ((uint32_t)f2bf(o[7]) << 16);
      *(uint4*)((uint16_t*)c + idx) = w;
    }
  }
};

// the buffer descriptor of a loader's tensor (BUF kernels; unused else)
template <class L, bool B>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const L& l) {
  if constexpr (B) return dma_rsrc(l.dbase());
  else return dma_rsrc(nullptr);
}

__device__ __forceinline__ int hk(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// W8: 8 waves (2 x 4, each 64 x BN/4) per 128 x BN block instead of 4 (2 x 2,
// each 64 x BN/2): twice the waves per CU at the same LDS footprint, for
// latency cover; LDS-DMA loaders only, BN 64 / 128.
// VAR: the part of the loaded 128 x BN tile the block computes (the LDS
// images and their DMA are those of the default tile in every variant):
//   0  all of it;
//   1  96 rows (8 waves as 2 x 4, 3 m-tiles of 16 each): an output of 96
//      rows (AlexNet conv1 weight gradient, OC = 96) wastes no MFMAs on the
//      zero rows 96..127 of the 128-row tile;
//   2  48 columns of a 64-wide tile (4 waves stacked along M, each 32 x 48):
//      a 48-wide output (AlexNet conv2 backward-data, 48 channels per group);
//   3  a 256-row tile (twice the A stage), 8 waves stacked along M, each
//      32 x BN (BN 64): narrow outputs move 0.83x the L2 -> LDS bytes per
//      FLOP of the 128 x 64 tile and still fit two blocks per CU (80 KiB);
//   4  as 3, computing 48 of the 64 columns.
// ABL (diagnostic builds only, selected by hvk_set_gemm_variant 11..13 in
// A/B runs; wrong results by design): 1 half the MFMAs (ks = 0 only), 2 no
// LDS-DMA after the first K tile, 3 neither DMA nor barriers after it.
template <class LA, bool AK, class LB, bool BKM, int BN_, bool BUF, bool W8,
          int VAR = 0, int ABL = 0>
__global__ void __launch_bounds__(W8 ? 512 : NTHR, 2)
gemm_kernel(LA la, LB lb, Epi epi, int M, int N, int K, int k_split,
            int tiles_n, int tiles, int splits, int gm) {
  constexpr int NW = W8 ? 8 : 4;        // waves per block
  constexpr int NT = NW * 64;           // threads per block
  constexpr int BMT = VAR >= 3 ? 256 : BM;     // rows loaded per block
  constexpr int WNC = VAR >= 2 ? 1 : NW / 2;   // waves along N
  constexpr int MT = VAR == 1 ? 3 : (VAR >= 2 ? 2 : 4);  // m-tiles per wave
  constexpr int WMR = 16 * MT;                 // rows per wave
  constexpr int BMC = (NW / WNC) * WMR;        // rows computed per block
  constexpr int NC = (VAR == 2 || VAR == 4) ? 48 : BN_;  // columns computed
  constexpr int NB = NC / (16 * WNC);          // MFMA n-tiles per wave
  static_assert(BMC <= BMT && NC <= BN_ && NB * 16 * WNC == NC, "layout");
  static_assert(!W8 || BN_ % 64 == 0, "W8 needs BN 64 / 128");
  static_assert(VAR < 3 || (W8 && AK && BKM && BN_ == 64 && BMC == 256),
                "256-row tiles: 8 waves, K-major operands, BN 64");
  constexpr int CPR = BN_ / 8;          // MN-major B: chunks per k-row
  constexpr int RPS = NTHR / CPR;       // MN-major B: k-rows per sweep
  // operand double buffers (64 KiB); reused as the f32 C tile (with a
  // 4-float row pad) by the epilogue
  // A stages (BM x BK) then B stages (BN x BK K-major, or the 128-wide
  // MN-major image); a 64-wide K-major B halves its stage, so such kernels
  // fit 3 blocks per CU (48 KiB) instead of 2
  constexpr int SA = BMT * BK;
  constexpr int SB = (BKM ? BN_ : 128) * BK;
  constexpr int SMEM_BYTES = (2 * (SA + SB) * 2 > BMT * (BN_ + 4) * 4)
                                 ? 2 * (SA + SB) * 2 : BMT * (BN_ + 4) * 4;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM_BYTES / 2];
  // 1-D grid over (group, split, tile), tile fastest.  Bijective XCD remap
  // (cdna_hip_programming.md T1): each XCD gets a contiguous wgid range, so
  // the tiles of one K split (which share the A rows / B columns of that
  // split) and neighbouring output tiles share one L2.
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gs = wgid / tiles;
  const int gi = gs / splits;
  // grouped tile order: runs of gm tile rows, column-major inside a run, so
  // the ~64 blocks an XCD holds at once cover a gm x (64 / gm) patch of C
  // and share both their A rows and their B columns in its L2 (row-major,
  // the 64 blocks share one A row and 64 B columns that stream from MALL)
  int tm, tn;
  if (gm > 1) {
    const int tiles_m = tiles / tiles_n;
    const int g = tile / (gm * tiles_n);
    const int m0g = g * gm;
    const int gh = min(tiles_m - m0g, gm);
    const int r = tile - g * gm * tiles_n;
    tm = m0g + r % gh;
    tn = r / gh;
  } else {
    tm = tile / tiles_n;
    tn = tile - tm * tiles_n;
  }
  const int split = gs - gi * splits;
  const int kbeg = split * k_split;
  const int kend = min(K, kbeg + k_split);
  if (kbeg >= kend) return;
  la.group(gi);
  lb.group(gi);
  const int m0 = tm * BMC, n0 = tn * NC;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WNC, wn = wid % WNC;

  const int fr = lane & 15, fq = lane >> 4;
  const int trq = fr >> 2, trp = fr & 3;
  f32x4 acc[MT][NB];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto frag_k = [&](const uint16_t* s, int rowbase, int ks) -> bf16x8 {
    int row = rowbase + fr;
    int c = ks * 4 + fq;
    return *(const bf16x8*)(s + row * 64 + ((c ^ (row & 7)) << 3));
  };
  auto frag_mn = [&](const uint16_t* s, int colbase, int ks) -> bf16x8 {
    int k = ks * 32 + fq * 8 + trq;
    int b = colbase >> 4;  // 32-B block of this 16-col tile
    const uint16_t* p0 = s + k * 128 + ((b ^ hk(k)) << 4) + trp * 4;
    const uint16_t* p1 = s + (k + 4) * 128 + ((b ^ hk(k + 4)) << 4) + trp * 4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  };
  auto compute = [&](const uint16_t* sA, const uint16_t* sB) {
#pragma unroll
    for (int ks = 0; ks < (ABL == 1 ? 1 : 2); ++ks) {
      bf16x8 af[MT], bfv[NB];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if constexpr (AK) af[i] = frag_k(sA, wm * WMR + i * 16, ks);
        else af[i] = frag_mn(sA, wm * WMR + i * 16, ks);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if constexpr (BKM) bfv[i] = frag_k(sB, wn * (NC / WNC) + i * 16, ks);
        else bfv[i] = frag_mn(sB, wn * (NC / WNC) + i * 16, ks);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfv[j],
                                                              acc[i][j], 0, 0, 0);
    }
  };
  const int nk = (kend - kbeg + BK - 1) / BK;

  bool done = false;
  constexpr bool GL = LA::kGlds && LB::kGlds;
  if constexpr (GL) {
    if (la.dma_ok() && lb.dma_ok()) {
      // ---- LDS-DMA pipeline (global_load_lds_dwordx4): the next tile's
      // loads stay in flight across the barrier; one counted vmcnt per tile.
      constexpr int NIA = BMT / 8 / NW;    // DMA instructions / wave (A)
      constexpr int NIB = BKM ? BN_ / (8 * NW) : 16 / NW;
      const int w = __builtin_amdgcn_readfirstlane(wid);
      typename LA::Ctx da[NIA];
      DRow fa[NIA];  // fast A loaders (K-major): per-slot row state
      typename LB::Ctx db[NIB];
      constexpr bool FB = !BKM && LB::kFast;  // fast MN-major B (wgrad)
      typename DColOf<LB, FB>::type fb[NIB];
      int ka[NIA], kb[NIB];
      // the lane's chunk offset along K: the same in every A slot
      const int kc = 8 * ((lane & 7) ^ ((lane >> 3) & 7));
      // BUF (loaders with kBuf, tensors < 2 GiB): LDS-DMA through buffer
      // descriptors - a per-slot 32-bit byte offset instead of a 64-bit
      // address, and kBufOOB lanes read zeros (no zero-page select)
      // per operand: BUF kernels use buffers for every loader that can
      constexpr bool BA = BUF && LA::kBuf, BB = BUF && LB::kBuf;
      const __amdgpu_buffer_rsrc_t ra = rsrc_of<LA, BA>(la);
      const __amdgpu_buffer_rsrc_t rb = rsrc_of<LB, BB>(lb);
      uint32_t va[NIA], vb[NIB];
      // MN-major B at BN = 64: the DMA image keeps the 256-B rows of the
      // 128-wide layout; the chunks of columns >= 64 read the zero page
      bool bz[NIB];
#pragma unroll
      for (int i = 0; i < NIA; ++i) {
        const int I = w * NIA + i;
        if constexpr (AK && LA::kFast) {
          fa[i] = la.drow(m0 + 8 * I + (lane >> 3));
          ka[i] = kc;
        } else if constexpr (AK && BA) {
          va[i] = la.row_voff(m0 + 8 * I + (lane >> 3));
          ka[i] = kc;
        } else if constexpr (AK) {
          int row = 8 * I + (lane >> 3);
          int c = (lane & 7) ^ ((lane >> 3) & 7);
          da[i] = la.row_ctx(m0 + row);
          ka[i] = 8 * c;
        } else {
          int hkv = ((lane >> 4) & 3) | (((I >> 1) & 1) << 2);
          int c = ((((lane & 15) >> 1) ^ hkv) << 1) | (lane & 1);
          ka[i] = 4 * I + (lane >> 4);
          if constexpr (BA)
            va[i] = la.col_voff(m0 + 8 * c, ka[i]);
          else
            da[i] = la.col_ctx(m0 + 8 * c);
        }
      }
#pragma unroll
      for (int i = 0; i < NIB; ++i) {
        const int I = w * NIB + i;
        if constexpr (BKM && BB) {
          vb[i] = lb.row_voff(n0 + 8 * I + (lane >> 3));
          kb[i] = kc;
        } else if constexpr (BKM) {
          int row = 8 * I + (lane >> 3);
          int c = (lane & 7) ^ ((lane >> 3) & 7);
          db[i] = lb.row_ctx(n0 + row);
          kb[i] = 8 * c;
        } else {
          int hkv = ((lane >> 4) & 3) | (((I >> 1) & 1) << 2);
          int c = ((((lane & 15) >> 1) ^ hkv) << 1) | (lane & 1);
          bz[i] = BN_ < 128 && 8 * c >= BN_;
          kb[i] = 4 * I + (lane >> 4);
          if constexpr (FB)
            fb[i] = lb.dcol(n0 + 8 * c, kbeg + kb[i], bz[i]);
          else if constexpr (BB)
            vb[i] = bz[i] ? kBufOOB : lb.col_voff(n0 + 8 * c, kb[i]);
          else
            db[i] = lb.col_ctx(n0 + (bz[i] ? 0 : 8 * c));
        }
        if constexpr (BKM) bz[i] = false;
      }
      auto issue = [&](int k0, uint16_t* sA, uint16_t* sB) {
        // the K-major lanes' byte offset along K and its validity (BUF)
        const uint32_t kbyte = 2u * (uint32_t)(k0 + kc);
        if constexpr (AK && LA::kFast && BA) {
          const DTap tp = la.dtap(k0 + kc);
#pragma unroll
          for (int i = 0; i < NIA; ++i)
            dma16(ra, sA + (w * NIA + i) * 512, la.dvoff(fa[i], tp));
        } else if constexpr (AK && BA) {
          const bool kin = k0 + kc < la.K;
#pragma unroll
          for (int i = 0; i < NIA; ++i)
            dma16(ra, sA + (w * NIA + i) * 512, kin ? va[i] + kbyte : kBufOOB);
        } else if constexpr (AK && LA::kFast) {
          const DTap tp = la.dtap(k0 + kc);
#pragma unroll
          for (int i = 0; i < NIA; ++i)
            __builtin_amdgcn_global_load_lds(
                (const void*)la.dsrc(fa[i], tp),
                (__attribute__((address_space(3))) void*)(sA + (w * NIA + i) * 512),
                16, 0, 0);
        } else if constexpr (!AK && BA) {
          // MN-major: the k-row advance is one uniform byte offset per tile
          const uint32_t kadv = (uint32_t)k0 * (uint32_t)la.ld * 2u;
#pragma unroll
          for (int i = 0; i < NIA; ++i)
            dma16(ra, sA + (w * NIA + i) * 512,
                  k0 + ka[i] < la.K ? va[i] + kadv : kBufOOB);
        } else {
#pragma unroll
          for (int i = 0; i < NIA; ++i)
            __builtin_amdgcn_global_load_lds(
                (const void*)la.src(da[i], k0 + ka[i]),
                (__attribute__((address_space(3))) void*)(sA + (w * NIA + i) * 512),
                16, 0, 0);
        }
        if constexpr (BKM && BB) {
          const bool kin = k0 + kc < lb.K;
#pragma unroll
          for (int i = 0; i < NIB; ++i)
            dma16(rb, sB + (w * NIB + i) * 512, kin ? vb[i] + kbyte : kBufOOB);
        } else if constexpr (!BKM && BB) {
          const uint32_t kadv = (uint32_t)k0 * (uint32_t)lb.ld * 2u;
#pragma unroll
          for (int i = 0; i < NIB; ++i)
            dma16(rb, sB + (w * NIB + i) * 512,
                  k0 + kb[i] < lb.K ? vb[i] + kadv : kBufOOB);
        } else if constexpr (FB) {
          // k0 advances by BK per call: the slot state tracks it
#pragma unroll
          for (int i = 0; i < NIB; ++i) {
            __builtin_amdgcn_global_load_lds(
                (const void*)lb.dsrc(fb[i]),
                (__attribute__((address_space(3))) void*)(sB + (w * NIB + i) * 512),
                16, 0, 0);
            lb.dnext(fb[i]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NIB; ++i)
            __builtin_amdgcn_global_load_lds(
                (const void*)(bz[i] ? g_zero8 : lb.src(db[i], k0 + kb[i])),
                (__attribute__((address_space(3))) void*)(sB + (w * NIB + i) * 512),
                16, 0, 0);
        }
      };
      issue(kbeg, smem, smem + 2 * SA);
      for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk && ABL < 2) {
          issue(kbeg + (kt + 1) * BK, smem + (cur ^ 1) * SA,
                smem + 2 * SA + (cur ^ 1) * SB);
          // leave exactly the next tile's DMAs (NIA + NIB) in flight
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIA + NIB) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (ABL < 3 || kt == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        compute(smem + cur * SA, smem + 2 * SA + cur * SB);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ABL < 3) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      done = true;
    }
  }
  if constexpr (!W8) if (!done) {
  typename LA::Ctx ca[4];
  typename LB::Ctx cb[4];
  if constexpr (AK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) ca[i] = la.row_ctx(m0 + (t >> 3) + 32 * i);
  } else {
    ca[0] = la.col_ctx(m0 + (t & 15) * 8);
  }
  if constexpr (BKM) {
#pragma unroll
    for (int i = 0; i < NB; ++i) cb[i] = lb.row_ctx(n0 + (t >> 3) + 32 * i);
  } else {
    cb[0] = lb.col_ctx(n0 + (t % CPR) * 8);
  }

  uint4 ra[4], rb[NB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (AK) ra[i] = la.load(ca[i], k0 + (t & 7) * 8);
      else ra[i] = la.load(ca[0], k0 + (t >> 4) + 16 * i);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (BKM) rb[i] = lb.load(cb[i], k0 + (t & 7) * 8);
      else rb[i] = lb.load(cb[0], k0 + t / CPR + RPS * i);
    }
  };
  auto sstore = [&](uint16_t* sA, uint16_t* sB) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (AK) {
        int row = (t >> 3) + 32 * i, c = t & 7;
        *(uint4*)(sA + row * 64 + ((c ^ (row & 7)) << 3)) = ra[i];
      } else {
        int k = (t >> 4) + 16 * i, c = t & 15;
        *(uint4*)(sA + k * 128 + (((c >> 1) ^ hk(k)) << 4) + ((c & 1) << 3)) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (BKM) {
        int row = (t >> 3) + 32 * i, c = t & 7;
        *(uint4*)(sB + row * 64 + ((c ^ (row & 7)) << 3)) = rb[i];
      } else {
        int k = t / CPR + RPS * i, c = t % CPR;
        *(uint4*)(sB + k * 128 + (((c >> 1) ^ hk(k)) << 4) + ((c & 1) << 3)) = rb[i];
      }
    }
  };

  gload(kbeg);
  sstore(smem, smem + 2 * SA);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) gload(kbeg + (kt + 1) * BK);
    compute(smem + cur * SA, smem + 2 * SA + cur * SB);
    if (more) sstore(smem + (cur ^ 1) * SA, smem + 2 * SA + (cur ^ 1) * SB);
    __syncthreads();
    cur ^= 1;
  }
  }  // register-staged path

  if (epi.atomic) {
    // split-K partial sums: f32 atomics straight from the accumulators
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        int mb = m0 + wm * WMR + i * 16 + fq * 4;
        int n = n0 + wn * (NC / WNC) + j * 16 + fr;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) epi.store(gi, mb + rr, n, acc[i][j][rr]);
      }
    return;
  }
  // stage the f32 tile through LDS, then row-contiguous 16-B stores
  constexpr int LDC = BN_ + 4;
  float* sC = (float*)smem;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int rb = wm * WMR + i * 16 + fq * 4;
      int cc = wn * (NC / WNC) + j * 16 + fr;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sC[(rb + rr) * LDC + cc] = acc[i][j][rr];
    }
  __syncthreads();
  constexpr int CH = NC / 8;
  const bool fast = epi.fast_ok();
  const float qs = epi.q8.q ? fp8_scale(epi.q8.st, epi.q8.hist, epi.q8.fmax)
                            : 1.f;
  float amax = 0.f;
  const int eg = epi.slice ? split : gi;  // row-offset index of the store
  for (int q = t; q < BMC * CH; q += NT) {
    int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
    if (m0 + row >= M) continue;
    const float4* src = (const float4*)(sC + row * LDC + c8);
    float v[8];
    float4 lo = src[0], hi = src[1];
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    if (fast && n0 + c8 + 8 <= epi.N &&
        (epi.ones_col < 0 || n0 + c8 + 8 <= epi.ones_col))
      epi.store8_fast(eg, m0 + row, n0 + c8, v, qs, &amax);
    else
      epi.store8(eg, m0 + row, n0 + c8, v);
  }
  if (epi.q8.q) {  // block-uniform
    __syncthreads();   // sC reads done: its first words hold the reduction
    q8_block_amax(epi.q8, amax, sC);
  }
}

#include "gemm_pp.h"
#include "gemm_t4.h"

// Tile width: 128 unless it wastes more than 1/8 of the columns; then 64,
// or 96 for a single 96-wide column tile (K-major B only: AlexNet conv1,
// N = 96, +16 % over 128).  N = 192 measured faster as 3 x 64 than as
// 2 x 96 (conv4 fwd 598 vs 536 TF: the 96 tile holds 150+ VGPRs).  Wide N
// keeps 128 so the A operand is re-read by as few column tiles as possible.
// The 128 tile is kept while it wastes at most N / div columns: div = 8 for
// K-major B, 2 for MN-major B - a 64-wide MN-major B tile still DMAs the
// 128-wide image (the upper half from the zero page), so it saves no fill
// bandwidth and only adds tiles (AlexNet conv1 wgrad, N = 432: 126 -> 203 TF
// at 128, step +1.5 %; profiles/gemm_experiments_r1.md §4).
inline int bn_waste_div(bool kmajor) { return kmajor ? 8 : 2; }
inline int pick_bn(int N, bool allow96) {
  auto waste = [&](int b) { return (N + b - 1) / b * b - N; };
  if (waste(128) * bn_waste_div(allow96) <= N) return 128;
  int best = 128;
  if (allow96 && N <= 96 && waste(96) < waste(best)) best = 96;
  if (waste(64) < waste(best)) best = 64;
  return best;
}

// GEMM schedule selector hvk_gemm_variant (A/B experiments set it through
// hvk_set_gemm_variant; nothing is read from the environment): 0 = 4-wave
// blocks everywhere,
// default (-1) = 8-wave blocks for the LDS-DMA loaders at BN 64 / 128
// except conv backward-data.  Measured on
// the AlexNet / VGG shapes (profiles/gemm_experiments_r2.md §6): 8 waves
// per block (4 per SIMD) lift the weight gradients 9-13 % and the FC GEMMs
// 4-7 %, the forward convs 0-4 %; backward-data loses 1-2 %.

template <class LA, class LB>
bool want_w8(const LA& la, const LB& lb, int bn) {
  const int v = hvk_gemm_variant;
  if (v == 0 || !(LA::kGlds && LB::kGlds) || (bn != 64 && bn != 128) ||
      !la.dma_ok() || !lb.dma_ok())
    return false;
  return v == 1 || !std::is_base_of<ConvDgradA, LA>::value;
}

// one kernel instantiation
template <class LA, bool AK, class LB, bool BKM, int BN_, bool BUF, bool W8,
          int VAR = 0>
hipError_t go(const LA& la, const LB& lb, const Epi& epi, int M, int N, int K,
              int k_split, int tiles_n, int tiles, int splits, dim3 grid,
              hipStream_t s) {
  // grouped tile order (8 tile rows per run) for C at least 8 tiles wide;
  // hvk_gemm_variant 20 keeps row-major (A/B runs)
  const int gm = (tiles_n >= 8 && hvk_gemm_variant != 20) ? 8 : 1;
  if constexpr (W8 && BN_ == 128 && VAR == 0 && BUF && AK && BKM &&
                std::is_same<LB, DenseK>::value &&
                (std::is_same<LA, DenseK>::value ||
                 std::is_same<LA, ConvFwdA>::value)) {
    const int v = hvk_gemm_variant;
    if (v >= 11 && v <= 13) {
      auto k = v == 11 ? gemm_kernel<LA, AK, LB, BKM, BN_, BUF, W8, 0, 1>
             : v == 12 ? gemm_kernel<LA, AK, LB, BKM, BN_, BUF, W8, 0, 2>
                       : gemm_kernel<LA, AK, LB, BKM, BN_, BUF, W8, 0, 3>;
      hipLaunchKernelGGL(k, grid, dim3(512), 0, s, la, lb, epi, M, N, K,
                         k_split, tiles_n, tiles, splits, gm);
      return launch_status(s);
    }
  }
  hipLaunchKernelGGL((gemm_kernel<LA, AK, LB, BKM, BN_, BUF, W8, VAR>), grid,
                     dim3(W8 ? 512 : NTHR), 0, s, la, lb, epi, M, N, K,
                     k_split, tiles_n, tiles, splits, gm);
  return launch_status(s);
}

template <class LA, bool AK, class LB, bool BKM, bool BUF>
hipError_t launch_bn(const LA& la, const LB& lb, const Epi& epi, int M, int N,
                     int K, int k_split, int tiles_n, int tiles, int splits,
                     int bn, dim3 grid, hipStream_t s) {
  // implicit-GEMM convolution forward / backward-data with >= 256 output
  // channels per group (VGG conv3-5, AlexNet conv3 backward-data): the
  // 256 x 256 ping-pong loop, 0.0078 operand bytes per FLOP against the T4
  // loop's 0.013 (gemm_pp.h).  Default settings only (any A/B variant keeps
  // them on T4 / the 128-row loop); hvk_gemm_variant 56 takes it for every
  // conv with >= 256 outputs per group (tests)
  if constexpr (BUF && AK && BKM && std::is_same<LB, DenseK>::value &&
                (std::is_same<LA, ConvFwdA>::value ||
                 std::is_same<LA, ConvDgradA>::value)) {
    const int groups = (int)(grid.x / ((unsigned)tiles * splits));
    // long reductions only (K >= 3072): AlexNet conv3 backward-data (K =
    // 3456) 996 -> 1067 TF, VGG conv3_2 (K = 2304) 987 -> 902 forward
    const bool force = hvk_gemm_variant == 56 && N >= 256;
    if ((hvk_gemm_variant < 0 || force) && splits == 1 && !epi.atomic &&
        !epi.slice && la.dma_ok() && lb.dma_ok() &&
        (force || (K >= 3072 && want_pp256(M, N, 1, groups))))
      return go_pp256<LA, AK, LB, BKM>(la, lb, epi, M, N, K, k_split, 1,
                                       groups, s);
  }
  // conv weight gradients with >= 256 output channels per group (VGG
  // conv3-5): the 256 x 256 ping-pong loop with the MN-major dY and im2col
  // loaders, split over pixels as the 128-row loop.  Opt-in
  // (hvk_gemm_variant 63): VGG conv3_2 at b1024 ran 820 -> 666 TF on it,
  // the VGG-16 b512 step 8.06k -> 7.88k img/s
  // (profiles/r4/t4_ablation/ab_pp256_wgrad.log)
  if constexpr (!AK && !BKM && std::is_same<LA, DenseMN>::value &&
                std::is_same<LB, ConvWgradB>::value) {
    const int groups = (int)(grid.x / ((unsigned)tiles * splits));
    const int wm = (M + 255) / 256 * 256 - M;
    if (hvk_gemm_variant == 63 && M >= 256 && wm * 8 <= M && epi.atomic &&
        !epi.slice && la.dma_ok() && lb.dma_ok() && lb.g.OH * lb.g.OW >= 64) {
      const long long pt = (long long)((M + 255) / 256) * ((N + 255) / 256);
      const long long want = ((long long)tiles * splits + pt - 1) / pt;
      int ks = (int)((K + want - 1) / want);
      ks = (ks + BK - 1) / BK * BK;
      const int sp = (K + ks - 1) / ks;
      return go_pp256<LA, AK, LB, BKM>(la, lb, epi, M, N, K, ks, sp, groups,
                                       s);
    }
  }
  // TN GEMMs without the bias-gradient ones column (FC weight gradients
  // whose bias gradient is a separate col_sum, engine.fc_bias_colsum):
  // both operands MN-major, the 256 x 256 loop where want_pp256 takes it;
  // a split-K accumulation is re-split as the 256 x 128 path below does.
  // hvk_gemm_variant 64 turns it off (A/B runs)
  if constexpr (BUF && !AK && !BKM && std::is_same<LA, DenseMN>::value &&
                std::is_same<LB, DenseMN>::value) {
    const int groups = (int)(grid.x / ((unsigned)tiles * splits));
    if (hvk_gemm_variant != 64 && groups == 1 && !epi.slice &&
        epi.ones_col < 0 && la.dma_ok() && lb.dma_ok()) {
      int sp = splits, ks = k_split;
      if (epi.atomic == 1 && splits > 1) {
        const long long pt = (long long)((M + 255) / 256) * ((N + 255) / 256);
        const long long want = ((long long)tiles * splits + pt - 1) / pt;
        ks = (int)((K + want - 1) / want);
        ks = (ks + BK - 1) / BK * BK;
        sp = (K + ks - 1) / ks;
      }
      if ((epi.atomic == 1 || sp == 1) && want_pp256(M, N, sp, 1))
        return go_pp256<LA, AK, LB, BKM>(la, lb, epi, M, N, K, ks, sp, 1, s);
    }
  }
  // implicit-GEMM convolutions: 192 x 128 tiles, two workgroups per CU
  // (gemm_t4.h)
  if constexpr (BUF && t4_pair_ok<LA, AK, LB, BKM>()) {
    const int groups = (int)(grid.x / ((unsigned)tiles * splits));
    bool taken = false;
    const hipError_t r = t4_launch<LA, AK, LB, BKM>(
        la, lb, epi, M, N, K, k_split, tiles, splits, groups, bn, s, &taken);
    if (taken) return r;
  }
  // large dense NT / NN GEMMs: the ping-pong 256 x 128 loop (gemm_pp.h)
  if constexpr (BUF && pp_loader_ok<LA, AK, true>() &&
                pp_loader_ok<LB, BKM, false>()) {
    const int groups = (int)(grid.x / ((unsigned)tiles * splits));
    // a split-K accumulation (f32 atomics) is re-split so that the 256 x 128
    // tiles launch as many workgroups as the 128 x bn tiles would have
    int sp = splits, ks = k_split;
    if (epi.atomic == 1 && splits > 1) {
      const long long pt = (long long)((M + PP_BM - 1) / PP_BM) *
                           ((N + PP_BN - 1) / PP_BN);
      const long long want = ((long long)tiles * splits + pt - 1) / pt;
      ks = (int)((K + want - 1) / want);
      ks = (ks + BK - 1) / BK * BK;
      sp = (K + ks - 1) / ks;
    }
    if (!epi.slice && want_pp<LA, AK, LB, BKM>(la, lb, M, N, bn, sp, groups))
      return go_pp<LA, AK, LB, BKM>(la, lb, epi, M, N, K, ks, sp, groups, s);
  }
#define HVK_GO(BNV, W8V, VARV)                                              \
  return go<LA, AK, LB, BKM, BNV, BUF, W8V, VARV>(la, lb, epi, M, N, K,     \
                                                  k_split, tiles_n, tiles,  \
                                                  splits, grid, s)
  // narrow K-major GEMMs (64-wide column tiles: conv backward-data with 48 /
  // 192 channels per group, forward with 192 outputs per group) over many
  // rows: the 256-row tile (VAR 3 / 4); hvk_gemm_variant 40 turns it off
  if constexpr (AK && BKM && LA::kGlds && LB::kGlds) {
    if (bn == 64 && hvk_gemm_variant != 40 && hvk_gemm_variant != 0 &&
        la.dma_ok() && lb.dma_ok()) {
      const int groups = (int)(grid.x / ((unsigned)tiles * splits));
      const int t256 = (M + 255) / 256 * tiles_n;
      if ((long long)t256 * splits * groups >= 512) {
        const dim3 g256((unsigned)((long long)t256 * splits * groups));
        if (N > 32 && N <= 48)
          return go<LA, AK, LB, BKM, 64, BUF, true, 4>(
              la, lb, epi, M, N, K, k_split, tiles_n, t256, splits, g256, s);
        return go<LA, AK, LB, BKM, 64, BUF, true, 3>(
            la, lb, epi, M, N, K, k_split, tiles_n, t256, splits, g256, s);
      }
    }
  }
  // (backward-data never runs 8-wave: not instantiated, half the compile)
  if constexpr (LA::kGlds && LB::kGlds &&
                !std::is_base_of<ConvDgradA, LA>::value) {
    if (want_w8(la, lb, bn)) {
      if constexpr (!AK && !BKM) {
        // 65..96 output rows: compute 96 of the 128 loaded (tiles_m is 1
        // either way)
        if (bn == 128 && M > 64 && M <= 96) HVK_GO(128, true, 1);
      }
      if (bn == 64) HVK_GO(64, true, 0);
      HVK_GO(128, true, 0);
    }
  }
  if constexpr (BKM && LA::kGlds && LB::kGlds &&
                std::is_base_of<ConvDgradA, LA>::value) {
    // 33..48 output columns per group (tiles_n is 1 either way): compute 48
    // of the 64 loaded; DMA loaders only (the variant has no register path)
    if (bn == 64 && N > 32 && N <= 48 && la.dma_ok() && lb.dma_ok())
      HVK_GO(64, false, 2);
  }
  if (bn == 64) HVK_GO(64, false, 0);
  if constexpr (BKM) {
    if (bn == 96) HVK_GO(96, false, 0);
  }
  HVK_GO(128, false, 0);
#undef HVK_GO
}

template <class LA, bool AK, class LB, bool BKM>
hipError_t launch_sel(const LA& la, const LB& lb, const Epi& epi, int M,
                      int N, int K, int k_split, int tiles_n, int tiles,
                      int splits, int groups, int bn, dim3 grid,
                      hipStream_t s);

template <class LA, bool AK, class LB, bool BKM>
hipError_t launch(const LA& la, const LB& lb, const Epi& epi, int M, int N,
                  int K, int splits, int groups, hipStream_t s) {
  // a 96-wide MN-major B has no register-staged path (12 chunks per row)
  const int bn = pick_bn(N, BKM);
  int tiles_m = (M + BM - 1) / BM, tiles_n = (N + bn - 1) / bn;
  if (splits < 1) splits = 1;
  int k_split = (K + splits - 1) / splits;
  k_split = (k_split + BK - 1) / BK * BK;
  splits = (K + k_split - 1) / k_split;
  const int tiles = tiles_m * tiles_n;
  dim3 grid((unsigned)((long long)tiles * splits * groups));
  if (epi.atomic == 2 && splits == 1) {
    // gradient OVERWRITE (the step's only contribution to C): plain stores,
    // no read of C, the bias-gradient column stored too - the optimizer
    // then needs no zeroing pass over the gradient buffer
    Epi e = epi;
    e.atomic = 0;
    e.beta = 0.f;
    e.bias_store = 1;
    return launch_sel<LA, AK, LB, BKM>(la, lb, e, M, N, K, k_split, tiles_n,
                                       tiles, splits, groups, bn, grid, s);
  }
  if (epi.atomic == 2) {
    // overwrite with split-K: zero C (and the bias gradient), then add
    if (groups != 1) return hipErrorInvalidValue;
    const int ncols = epi.ones_col >= 0 ? epi.ones_col : epi.N;
    hipError_t z = hipMemset2DAsync(
        epi.c, (size_t)epi.ldc * (epi.out_f32 ? 4 : 2), 0,
        (size_t)ncols * (epi.out_f32 ? 4 : 2), (size_t)epi.M, s);
    if (z != hipSuccess) return z;
    if (epi.bias_grad) {
      z = hipMemsetAsync(epi.bias_grad, 0, (size_t)epi.M * 4, s);
      if (z != hipSuccess) return z;
    }
    Epi e = epi;
    e.atomic = 1;
    return launch_sel<LA, AK, LB, BKM>(la, lb, e, M, N, K, k_split, tiles_n,
                                       tiles, splits, groups, bn, grid, s);
  }
  if (epi.atomic && splits == 1) {
    // an unsplit accumulate writes every element once: read-modify-write in
    // the staged epilogue instead of one f32 atomic per element (the FC
    // weight gradients at batch 512 were bound by the atomic rate)
    Epi e = epi;
    e.atomic = 0;
    e.beta = 1.f;
    return launch_sel<LA, AK, LB, BKM>(la, lb, e, M, N, K, k_split, tiles_n,
                                       tiles, splits, groups, bn, grid, s);
  }
  return launch_sel<LA, AK, LB, BKM>(la, lb, epi, M, N, K, k_split, tiles_n,
                                     tiles, splits, groups, bn, grid, s);
}

template <class LA, bool AK, class LB, bool BKM>
hipError_t launch_sel(const LA& la, const LB& lb, const Epi& epi, int M,
                      int N, int K, int k_split, int tiles_n, int tiles,
                      int splits, int groups, int bn, dim3 grid,
                      hipStream_t s) {
  if constexpr (LA::kBuf || LB::kBuf) {
    if ((!LA::kBuf || la.buf_ok(groups)) && (!LB::kBuf || lb.buf_ok(groups)))
      return launch_bn<LA, AK, LB, BKM, true>(la, lb, epi, M, N, K, k_split,
                                              tiles_n, tiles, splits, bn,
                                              grid, s);
  }
  return launch_bn<LA, AK, LB, BKM, false>(la, lb, epi, M, N, K, k_split,
                                           tiles_n, tiles, splits, bn, grid,
                                           s);
}


Epi make_epi(void* c, int ldc, int M, int N, int out_f32, int atomic,
             float alpha, float beta, const float* bias, int bias_mode,
             int act, const void* aux, int ld_aux, int aux_act) {
  Epi e;
  e.c = c; e.ldc = ldc; e.M = M; e.N = N; e.out_f32 = out_f32;
  e.atomic = atomic; e.alpha = alpha; e.beta = beta; e.bias = bias;
  e.bias_mode = bias ? bias_mode : 0; e.act = act;
  e.aux = (const uint16_t*)aux; e.ld_aux = ld_aux; e.aux_act = aux_act;
  e.grow = 0; e.gcol = 0; e.preact = nullptr;
  e.ones_col = -1; e.bias_grad = nullptr; e.run_in = 0; e.run_out = 0;
  e.bias_store = 0;
  e.slice = 0;
  e.q8.q = nullptr;
  e.q8.st = nullptr;
  e.q8.shard = nullptr;
  e.q8.fmax = 1.f;
  e.q8.fmt = 0;
  e.q8.hist = 0;
  return e;
}

// [OC][KH][RUNP] run geometry of the small-channel paths
inline RunGeom make_run(const ConvGeom& g) {
  RunGeom r;
  r.RUN = g.KW * g.C;
  r.RUNP = (r.RUN + 7) / 8 * 8;
  r.fRUNP = make_fastdiv(r.RUNP);
  r.fC = make_fastdiv(g.C);
  r.total = (long long)g.N * g.H * g.W * g.C;
  return r;
}

}  // namespace
