// gemm_fp8.hip - FP8 (OCP e4m3 / e5m2) MFMA GEMM and implicit-GEMM
// convolution (forward and backward-data) for gfx950, plus the per-tensor
// delayed-scaling quantizers that feed them.
//
// Matrix core: v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales
// (E8M0 127 = 2^0).  Per MI355X_MICROARCH.md (Matrix cores) this form runs at
// twice the bf16 rate per clock; the non-scaled 16x16x32 fp8 form would only
// match bf16.  Per-tensor scales are applied once, in the epilogue.
//
// Tile: 128 x {128,64} x 128 (k in BYTES = fp8 elements), 4 waves (2x2), each
// wave 64 x BN/2 = 4 x BN/32 MFMA tiles; one MFMA consumes the whole 128-deep
// K tile.  A K-major LDS row is 128 B - byte-for-byte the layout of the bf16
// kernel's 64-wide K tile (gemm.hip) - so the same 16-B chunk XOR swizzle
// (chunk c at c ^ (row & 7)) keeps the LDS-DMA image lane-linear.  Operands
// move by global_load_lds_dwordx4 with the next tile in flight across the
// (raw) barrier, one counted vmcnt per tile.
//
// Operand lane map: lane l feeds row (l & 15) with the 16-B chunks
// q = l >> 4 and q + 4 (k = 16q .. 16q + 15 and 64 + 16q ..) of both A and
// B.  The k order inside an MFMA is a permutation shared by A and B, so the
// sum over k is the same whatever order the hardware assigns
// (tests/test_fp8.py checks it against fp32); this pair keeps the
// ds_read_b128 lane groups conflict-free, as the bf16 loop's fragments.
//
// Only K-major operands exist here (fp8 has no transposed LDS read that the
// bf16 MN-major path relies on), which covers conv forward (A = im2col(X),
// B = W[OC][K]), conv dgrad (A = gather(dY), B = W permuted to [C][K]) and
// the fully-connected forward.  Weight gradients and the fully-connected
// dgrad (whose fp8 B operand would be W^T) stay on the bf16 kernels
// (docs/OPS.md §FP8).
#include <type_traits>

#include "fp8_common.h"
#include "conv_geom.h"

using namespace hvk;

typedef __attribute__((ext_vector_type(8))) int i32x8;

// fp8 schedule selector for A/B runs (hvk_set_fp8_variant): 70 keeps dense
// GEMMs on the 128-row loop
int hvk_fp8_variant = -1;

namespace {

constexpr int BM = 128, BK = 128, NTHR = 256;

__device__ __attribute__((aligned(16))) const uint8_t g_zero16[16] = {0};

// scales, packs, the fused-quantisation output: fp8_common.h

// ----------------------------------------------------------------- loaders
struct Dense8 {
  const uint8_t* p;
  long long gstride;
  int rows, K, ld;
  struct Ctx { const uint8_t* row; int ok; };
  __device__ void group(int g) { p += (long long)g * gstride; }
  __device__ __forceinline__ Ctx row_ctx(int r) const {
    Ctx c;
    c.ok = r < rows;
    c.row = p + (long long)(c.ok ? r : 0) * ld;
    return c;
  }
  static constexpr bool kFast = false;
  __device__ __forceinline__ const uint8_t* src(const Ctx& c, int k) const {
    // bitwise condition + pinned address: no exec-mask branch per slot
    return pick_ptr(c.row + k, (c.ok != 0) & (k < K), g_zero16);
  }
  // buffer-descriptor DMA (the ping-pong loop): byte offset of row r
  bool buf_ok() const {
    return (long long)(rows - 1) * ld + K < kBufMaxBytes;
  }
  __device__ __forceinline__ uint32_t row_voff(int r) const {
    return r < rows ? (uint32_t)r * (uint32_t)ld : kBufOOB;
  }
};

// conv forward A: rows = output pixels (n, oh, ow), k = (kh, kw, c); a
// 16-byte chunk is 16 channels of one tap (Cg % 16 == 0)
struct ConvFwdA8 {
  const uint8_t* x;
  ConvGeom g;
  int M, K, coff;
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
  __device__ __forceinline__ const uint8_t* src(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return g_zero16;
    uint32_t t, ch, kh, kw;
    fdivmod(k, g.fCg, t, ch);
    fdivmod(t, g.fKW, kh, kw);
    int ih = c.ih0 + (int)kh, iw = c.iw0 + (int)kw;
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W)
      return g_zero16;
    return x + c.base + (ih * g.W + iw) * g.C + ch;
  }
  // branch-free DMA addressing (conv_geom.h), as the bf16 ConvFwdA
  static constexpr bool kFast = true;
  __device__ __forceinline__ DRow drow(int m) const {
    return fwd_drow(g, M, coff, m);
  }
  __device__ __forceinline__ DTap dtap(int k) const { return fwd_dtap(g, K, k); }
  __device__ __forceinline__ const uint8_t* dsrc(const DRow& r,
                                                 const DTap& t) const {
    return pick_ptr(x + (r.pix + t.off), tap_ok(r, t), g_zero16);
  }
};

// conv dgrad A: rows = input pixels (n, h, w), k = (kh, kw, oc) over dY
struct ConvDgradA8 {
  const uint8_t* dy;
  ConvGeom g;
  int M, K, coff;
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
  __device__ __forceinline__ const uint8_t* src(const Ctx& c, int k) const {
    if (!c.ok || k >= K) return g_zero16;
    uint32_t t, oc, kh, kw;
    fdivmod(k, g.fOCg, t, oc);
    fdivmod(t, g.fKW, kh, kw);
    int ohs = c.hp - (int)kh, ows = c.wp - (int)kw;
    if (ohs < 0 || ows < 0) return g_zero16;
    int oh = ohs, ow = ows;
    if (g.sy != 1 || g.sx != 1) {
      oh = (int)fdiv((uint32_t)ohs, g.fSy);
      ow = (int)fdiv((uint32_t)ows, g.fSx);
      if (oh * g.sy != ohs || ow * g.sx != ows) return g_zero16;
    }
    if (oh >= g.OH || ow >= g.OW) return g_zero16;
    return dy + c.base + (oh * g.OW + ow) * g.OC + oc;
  }
  // branch-free DMA addressing for stride 1 (strided: ConvDgradA8Str)
  static constexpr bool kFast = true;
  __device__ __forceinline__ DRow drow(int m) const {
    return dgrad_drow(g, M, coff, m);
  }
  __device__ __forceinline__ DTap dtap(int k) const {
    return dgrad_dtap(g, K, k);
  }
  __device__ __forceinline__ const uint8_t* dsrc(const DRow& r,
                                                 const DTap& t) const {
    return pick_ptr(dy + (r.pix + t.off), tap_ok(r, t), g_zero16);
  }
};

struct ConvDgradA8Str : ConvDgradA8 {
  static constexpr bool kFast = false;
};

// ---------------------------------------------------------------- epilogue
struct Epi8 {
  uint16_t* c;           // bf16 output
  int ldc, M, N;
  int grow_unused, gcol;  // per-group column offset
  const float* bias;     // per column (f32) or null
  int act;
  const uint16_t* aux;   // multiply by act_bwd(aux, aux_act)
  int ld_aux, aux_act;
  const float* sa;       // scaler states of A and B
  const float* sb;
  int hist;
  float fa, fb;          // effective fp8 maxima of A and B
  // fused quantisation for the NEXT fp8 op (optional): q8 (same indexing as
  // c) = sat(bf16(out) * scale(q8_st)) in format q8_fmt, and amax|bf16(out)|
  // into one of 32 shards of q8_shard (one atomicMax per workgroup; the
  // registry's roll folds the shards into the current amax)
  uint8_t* q8;
  const float* q8_st;
  float* q8_shard;
  float q8_fmax;
  int q8_fmt;
};

// the fused fp8 copy of 8 stored bf16 outputs: quantise what the consumer
// would read (the bf16-rounded values), amax of them into *amax
__device__ __forceinline__ void q8_out8(const Epi8& e, long long idx,
                                        const uint4& ob, float qs,
                                        float* amax) {
  const uint32_t w4[4] = {ob.x, ob.y, ob.z, ob.w};
  float r[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r[2 * q] = __uint_as_float(w4[q] << 16);
    r[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
  }
  const float lim = e.q8_fmt == 0 ? 448.f : 57344.f;
  float mx = *amax;
#pragma unroll
  for (int q = 0; q < 8; ++q) mx = fmaxf(mx, fabsf(r[q]));
  *amax = mx;
  uint2 qv;
  qv.x = pack4_fp8(sat(r[0] * qs, lim), sat(r[1] * qs, lim),
                   sat(r[2] * qs, lim), sat(r[3] * qs, lim), e.q8_fmt);
  qv.y = pack4_fp8(sat(r[4] * qs, lim), sat(r[5] * qs, lim),
                   sat(r[6] * qs, lim), sat(r[7] * qs, lim), e.q8_fmt);
  *(uint2*)(e.q8 + idx) = qv;
}

__device__ __forceinline__ void store8(const Epi8& e, float alpha, int gi,
                                       int m, int n, const float* v,
                                       float qs = 1.f, float* amax = nullptr) {
  if (m >= e.M || n >= e.N) return;
  const int gn = n + gi * e.gcol;
  const long long idx = (long long)m * e.ldc + gn;
  const bool vec = n + 8 <= e.N && (e.ldc & 7) == 0 && (gn & 7) == 0 &&
                   (!e.aux || (e.ld_aux & 7) == 0);
  float a[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = 1.f;
  if (e.aux) {
    if (vec) {
      uint4 av = *(const uint4*)(e.aux + (long long)m * e.ld_aux + gn);
      const uint16_t* ah = (const uint16_t*)&av;
      float y[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) y[q] = bf2f(ah[q]);
      act_bwd_mul8(a, y, e.aux_act);  // a = act_bwd(y), one switch
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (n + q < e.N)
          a[q] = act_bwd(bf2f(e.aux[(long long)m * e.ld_aux + gn + q]),
                         e.aux_act);
    }
  }
  float o[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = v[q] * alpha;
  if (e.bias) {
    if (vec && (((uintptr_t)(e.bias + gn)) & 15) == 0) {
      const float4 b0 = *(const float4*)(e.bias + gn);
      const float4 b1 = *(const float4*)(e.bias + gn + 4);
      o[0] += b0.x; o[1] += b0.y; o[2] += b0.z; o[3] += b0.w;
      o[4] += b1.x; o[5] += b1.y; o[6] += b1.z; o[7] += b1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (n + q < e.N) o[q] += e.bias[gn + q];
    }
  }
  // one switch per chunk (act_fwd8); a[] already holds act_bwd(aux)
  act_fwd8(o, e.act);
  if (e.aux) {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] *= a[q];
  }
  if (vec) {
    const uint4 ob = pack_bf16x8(o);
    *(uint4*)(e.c + idx) = ob;
    if (e.q8) q8_out8(e, idx, ob, qs, amax);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (n + q < e.N) e.c[idx + q] = f2bf(o[q]);
    if (e.q8) {
      const float lim = e.q8_fmt == 0 ? 448.f : 57344.f;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (n + q < e.N) {
          const float r = bf2f(f2bf(o[q]));
          *amax = fmaxf(*amax, fabsf(r));
          e.q8[idx + q] = (uint8_t)(pack4_fp8(sat(r * qs, lim), 0.f, 0.f, 0.f,
                                              e.q8_fmt) & 0xFF);
        }
    }
  }
}

// 4 consecutive columns of one row from a lane's accumulator quad (the T4
// loop's direct epilogue); the launch checked store4_ok: 4-aligned rows,
// columns and aux rows, a 16-B aligned bias, n % 4 == 0 and N % 4 == 0
__host__ __device__ __forceinline__ bool store4_ok(const Epi8& e) {
  return (e.ldc & 3) == 0 && (e.gcol & 3) == 0 && (e.N & 3) == 0 &&
         (!e.aux || (e.ld_aux & 3) == 0) &&
         (!e.bias || (((uintptr_t)e.bias) & 15) == 0);
}
__device__ __forceinline__ void store4(const Epi8& e, float alpha, int gi,
                                       int m, int n, const float* v,
                                       float qs, float* amax) {
  const int gn = n + gi * e.gcol;
  const long long idx = (long long)m * e.ldc + gn;
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = v[q] * alpha;
  if (e.bias) {
    const float4 b = *(const float4*)(e.bias + gn);
    o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w;
  }
  act_fwd_n<4>(o, e.act);
  if (e.aux) {
    const uint2 av = *(const uint2*)(e.aux + (long long)m * e.ld_aux + gn);
    const uint16_t* ah = (const uint16_t*)&av;
    float y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = bf2f(ah[q]);
    act_bwd_mul_n<4>(o, y, e.aux_act);
  }
  const uint2 ob = make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
  *(uint2*)(e.c + idx) = ob;
  if (e.q8) {
    // quantise what the consumer would read: the bf16-rounded output
    float r[4];
    r[0] = __uint_as_float(ob.x << 16);
    r[1] = __uint_as_float(ob.x & 0xffff0000u);
    r[2] = __uint_as_float(ob.y << 16);
    r[3] = __uint_as_float(ob.y & 0xffff0000u);
    const float lim = e.q8_fmt == 0 ? 448.f : 57344.f;
    float mx = *amax;
#pragma unroll
    for (int q = 0; q < 4; ++q) mx = fmaxf(mx, fabsf(r[q]));
    *amax = mx;
    *(uint32_t*)(e.q8 + idx) =
        pack4_fp8(sat(r[0] * qs, lim), sat(r[1] * qs, lim),
                  sat(r[2] * qs, lim), sat(r[3] * qs, lim), e.q8_fmt);
  }
}

// 4 consecutive columns of one row finished in registers and packed to
// bf16 (the T4 register epilogue): alpha, bias, activation, derivative of
// the layer below - store8's arithmetic per element
__device__ __forceinline__ uint2 pre4_8(const Epi8& e, float alpha, int gi,
                                        int m, int n, const float* v) {
  const int gn = n + gi * e.gcol;
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = v[q] * alpha;
  if (e.bias) {
    const float4 b = *(const float4*)(e.bias + gn);
    o[0] += b.x; o[1] += b.y; o[2] += b.z; o[3] += b.w;
  }
  float a[4] = {1.f, 1.f, 1.f, 1.f};
  if (e.aux) {
    const uint2 av = *(const uint2*)(e.aux + (long long)m * e.ld_aux + gn);
    float y[4];
    y[0] = __uint_as_float(av.x << 16);
    y[1] = __uint_as_float(av.x & 0xffff0000u);
    y[2] = __uint_as_float(av.y << 16);
    y[3] = __uint_as_float(av.y & 0xffff0000u);
    act_bwd_mul_n<4>(a, y, e.aux_act);   // a = act_bwd(y), as store8
  }
  act_fwd_n<4>(o, e.act);
  if (e.aux) {
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] *= a[q];
  }
  return make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
}
// the register epilogue applies: 8-aligned rows, columns and N, 4-aligned
// aux rows, a 16-B aligned bias
__host__ __device__ __forceinline__ bool regepi_ok(const Epi8& e) {
  return (e.ldc & 7) == 0 && (e.gcol & 7) == 0 && (e.N & 7) == 0 &&
         (((uintptr_t)e.c) & 15) == 0 && (!e.aux || (e.ld_aux & 3) == 0) &&
         (!e.bias || (((uintptr_t)e.bias) & 15) == 0);
}

// ------------------------------------------------------------------ kernel
// W8: 8 waves (2 x 4, each 64 x BN/4) instead of 4 (2 x 2) on the same tile
// and LDS footprint - more waves per SIMD for latency cover (the bf16
// kernel's measurement: profiles/gemm_experiments_r2.md §6).
template <class LA, class LB, int BN_, int FA, int FB, bool W8>
__global__ void __launch_bounds__(W8 ? 512 : NTHR, 2)
gemm_fp8_kernel(LA la, LB lb, Epi8 epi, int M, int N, int K, int tiles_n,
                int tiles) {
  constexpr int NW = W8 ? 8 : 4;          // waves per block
  constexpr int NT = NW * 64;
  constexpr int WNC = NW / 2;             // waves along N
  constexpr int NB = BN_ / (16 * WNC);    // MFMA n-tiles per wave
  constexpr int SA = BM * BK;             // bytes per A stage
  constexpr int SB = BN_ * BK;            // bytes per B stage
  constexpr int OPER = 2 * (SA + SB);
  constexpr int LDC = BN_ + 4;            // f32 C tile row pitch
  constexpr int CT = BM * LDC * 4;
  constexpr int SMEM = OPER > CT ? OPER : CT;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gi = wgid / tiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  la.group(gi);
  lb.group(gi);
  const int m0 = tm * BM, n0 = tn * BN_;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid / WNC, wn = wid % WNC;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 32 bytes of row (rowbase + fr): chunks fq and fq + 4 at their swizzled
  // slots (c ^ (row & 7)) of the 128-B row.  Which k a lane holds only has
  // to agree between A and B (the MFMA sums every product); this pair is
  // the bf16 loop's two 32-deep fragments, conflict-free per ds_read_b128
  // lane group (chunks 2fq, 2fq + 1 put two lanes of a group on one bank
  // slot)
  auto frag = [&](const uint8_t* s, int rowbase) -> i32x8 {
    const int row = rowbase + fr;
    const int sw = row & 7;
    const uint8_t* base = s + row * BK;
    uint4 lo = *(const uint4*)(base + ((fq ^ sw) << 4));
    uint4 hi = *(const uint4*)(base + (((fq + 4) ^ sw) << 4));
    i32x8 v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  auto compute = [&](const uint8_t* sA, const uint8_t* sB) {
    i32x8 af[4], bfv[NB];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(sA, wm * 64 + i * 16);
#pragma unroll
    for (int j = 0; j < NB; ++j) bfv[j] = frag(sB, wn * (BN_ / WNC) + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            af[i], bfv[j], acc[i][j], FA, FB, 0, 127, 0, 127);
  };

  // LDS-DMA issue map: instruction I of a stage covers rows 8I..8I+7; lane
  // -> row 8I + (lane >> 3), LDS slot (lane & 7) holds chunk slot ^ (row & 7)
  constexpr int NIA = SA / (NT * 16);     // 4 (2 at W8)
  constexpr int NIB = SB / (NT * 16);     // 4 (BN 128) or 2 (BN 64); half at W8
  const int w = __builtin_amdgcn_readfirstlane(wid);
  typename LA::Ctx da[NIA];
  DRow fa[NIA];  // fast A loaders: per-slot row state
  typename LB::Ctx db[NIB];
  int ka[NIA], kb[NIB];
  // the lane's chunk offset along K (row & 7 == (lane >> 3) & 7 in every slot)
  const int kc = 16 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
  for (int i = 0; i < NIA; ++i) {
    const int I = w * NIA + i;
    const int row = 8 * I + (lane >> 3);
    if constexpr (LA::kFast)
      fa[i] = la.drow(m0 + row);
    else
      da[i] = la.row_ctx(m0 + row);
    ka[i] = kc;
  }
#pragma unroll
  for (int i = 0; i < NIB; ++i) {
    const int I = w * NIB + i;
    const int row = 8 * I + (lane >> 3);
    db[i] = lb.row_ctx(n0 + row);
    kb[i] = 16 * ((lane & 7) ^ (row & 7));
  }
  auto issue = [&](int k0, uint8_t* sA, uint8_t* sB) {
    if constexpr (LA::kFast) {
      const DTap tp = la.dtap(k0 + kc);
#pragma unroll
      for (int i = 0; i < NIA; ++i)
        __builtin_amdgcn_global_load_lds(
            (const void*)la.dsrc(fa[i], tp),
            (__attribute__((address_space(3))) void*)(sA + (w * NIA + i) * 1024),
            16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < NIA; ++i)
        __builtin_amdgcn_global_load_lds(
            (const void*)la.src(da[i], k0 + ka[i]),
            (__attribute__((address_space(3))) void*)(sA + (w * NIA + i) * 1024),
            16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NIB; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)lb.src(db[i], k0 + kb[i]),
          (__attribute__((address_space(3))) void*)(sB + (w * NIB + i) * 1024),
          16, 0, 0);
  };

  const int nk = (K + BK - 1) / BK;
  issue(0, smem, smem + 2 * SA);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      issue((kt + 1) * BK, smem + (cur ^ 1) * SA, smem + 2 * SA + (cur ^ 1) * SB);
      // leave exactly the next tile's DMAs in flight
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIA + NIB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(smem + cur * SA, smem + 2 * SA + cur * SB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // per-tensor dequantisation: 1 / (sA * sB)
  const float alpha = 1.f / (fp8_scale(epi.sa, epi.hist, epi.fa) *
                             fp8_scale(epi.sb, epi.hist, epi.fb));
  float* sC = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int rb = wm * 64 + i * 16 + fq * 4;
      const int cc = wn * (BN_ / WNC) + j * 16 + fr;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) sC[(rb + rr) * LDC + cc] = acc[i][j][rr];
    }
  __syncthreads();
  constexpr int CH = BN_ / 8;
  const float qs = epi.q8 ? fp8_scale(epi.q8_st, epi.hist, epi.q8_fmax) : 1.f;
  float amax = 0.f;
  for (int q = t; q < BM * CH; q += NT) {
    const int row = q / CH, c8 = (q - row * CH) * 8;
    if (m0 + row >= M) continue;
    const float4* src = (const float4*)(sC + row * LDC + c8);
    float v[8];
    float4 lo = src[0], hi = src[1];
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    store8(epi, alpha, gi, m0 + row, n0 + c8, v, qs, &amax);
  }
  if (epi.q8) {
    // one atomicMax per workgroup, spread over 32 shards (128-B apart) so
    // that tens of thousands of workgroups do not serialise on one address
    amax = wave_max(amax);
    __syncthreads();   // sC reads done: reuse its first words
    float* red = (float*)smem;
    if (lane == 0) red[wid] = amax;
    __syncthreads();
    if (t == 0) {
      float mx = 0.f;
      for (int i = 0; i < NW; ++i) mx = fmaxf(mx, red[i]);
      if (mx > 0.f)
        atomicMax((unsigned int*)(epi.q8_shard + (blockIdx.x & 31) * 32),
                  __float_as_uint(mx));
    }
  }
}

// ---------------------------------------------------------------------------
// fp8 implicit-GEMM convolution on the bf16 T4 loop (gemm_t4.h): 192 x 128
// tiles, 4 waves (2 x 2, each 96 x 64), two 40-KiB LDS stages of a 128-byte
// K tile (= the bf16 loop's 64-element tile, byte for byte), TWO
// workgroups per CU, one barrier per K tile, the next tile's DMA in flight
// during the MFMAs.  Per K tile a wave issues 10 LDS-DMA pieces and 20
// fragment reads (32 B each: two ds_read_b128) against 24 MFMAs of
// 16x16x128 (32 cycles each, twice the bf16 work per cycle).  P = the
// implicit im2col / gathered-dY rows (fast DRow / DTap addressing), Q = the
// weights (Dense8).
//
// QR = 64 (outputs of 64 channels per group: VGG conv1_2 forward, conv1_2 /
// conv2_1 backward-data) takes PR = 256 rows and stacks the four waves
// along P (each 64 x 64, 16 MFMAs per K tile): the same 40-KiB stage.
//
// DIR: the direct epilogue - the MFMAs compute the transposed tile (same
// values), so a lane's accumulator quad is 4 consecutive output channels of
// one pixel and goes straight to global memory (no LDS staging).
template <class LP, int FA, int FB, int PR = 192, int QR = 128,
          int EP = 0>
__global__ void __launch_bounds__(256, 2)
gemm_t4_fp8_kernel(LP lp, Dense8 lq, Epi8 epi, int P, int Q, int K,
                   int tiles_q, int tiles, int gm) {
  static_assert((PR == 192 && QR == 128) || (PR == 256 && QR == 64),
                "tile shapes");
  constexpr bool STK = QR == 64;        // waves stacked along P
  constexpr int MI = STK ? PR / 64 : PR / 32;   // m-tiles per wave
  constexpr int NJ = 4;                         // n-tiles per wave (64 cols)
  constexpr int SP = PR * BK, SQ = QR * BK, SST = SP + SQ;   // bytes
  constexpr int NSP = PR / 8 / 4, NSQ = QR / 8 / 4;          // per wave
  constexpr int HP = PR / 2, LDC = QR + 4;
  static_assert(HP * LDC * 4 <= 2 * SST, "epilogue pass fits");
  static_assert(2 * 2 * SST <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * SST];
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gi = wgid / tiles;
  int tp, tq;
  if (gm > 1) {
    const int tiles_p = tiles / tiles_q;
    const int g = tile / (gm * tiles_q);
    const int p0g = g * gm;
    const int gh = min(tiles_p - p0g, gm);
    const int r = tile - g * gm * tiles_q;
    tp = p0g + r % gh;
    tq = r / gh;
  } else {
    tp = tile / tiles_q;
    tq = tile - tp * tiles_q;
  }
  lp.group(gi);
  lq.group(gi);
  const int p0 = tp * PR, q0 = tq * QR;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int prow = STK ? w * (PR / 4) : (w >> 1) * HP;
  const int qrow = STK ? 0 : (w & 1) * 64;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA slots: piece I = rows 8I .. 8I + 7 of the operand, lane -> row
  // 8I + (lane >> 3), chunk (lane & 7) ^ (row & 7)
  const int kc = 16 * ((lane & 7) ^ ((lane >> 3) & 7));
  DRow fa[NSP];
  typename Dense8::Ctx db[NSQ];
#pragma unroll
  for (int i = 0; i < NSP; ++i)
    fa[i] = lp.drow(p0 + 8 * (w * NSP + i) + (lane >> 3));
#pragma unroll
  for (int i = 0; i < NSQ; ++i)
    db[i] = lq.row_ctx(q0 + 8 * (w * NSQ + i) + (lane >> 3));
  auto issue = [&](int k0, uint8_t* sP) {
    const DTap tpk = lp.dtap(k0 + kc);
#pragma unroll
    for (int i = 0; i < NSP; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)lp.dsrc(fa[i], tpk),
          (__attribute__((address_space(3))) void*)(sP + (w * NSP + i) * 1024),
          16, 0, 0);
#pragma unroll
    for (int i = 0; i < NSQ; ++i)
      __builtin_amdgcn_global_load_lds(
          (const void*)lq.src(db[i], k0 + kc),
          (__attribute__((address_space(3))) void*)(sP + SP +
                                                    (w * NSQ + i) * 1024),
          16, 0, 0);
  };
  auto frag = [&](const uint8_t* sb, int rowbase) -> i32x8 {
    const int row = rowbase + fr;
    const int sw = row & 7;
    const uint8_t* base = sb + row * BK;
    const uint4 lo = *(const uint4*)(base + ((fq ^ sw) << 4));
    const uint4 hi = *(const uint4*)(base + (((fq + 4) ^ sw) << 4));
    i32x8 v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  const int nk = (K + BK - 1) / BK;
  issue(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int kt = 0; kt < nk; ++kt) {
    const uint8_t* sP = smem + (kt & 1) * SST;
    const uint8_t* sQ = sP + SP;
    // tile t + 1 into the stage tile t - 1 used (read before the barrier
    // that ended step t - 1)
    if (kt + 1 < nk) issue((kt + 1) * BK, smem + ((kt + 1) & 1) * SST);
    i32x8 bq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bq[j] = frag(sQ, qrow + j * 16);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const i32x8 a = frag(sP, prow + i * 16);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (EP != 0)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              bq[j], a, acc[i][j], FB, FA, 0, 127, 0, 127);
        else
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              a, bq[j], acc[i][j], FA, FB, 0, 127, 0, 127);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  const float alpha = 1.f / (fp8_scale(epi.sa, epi.hist, epi.fa) *
                             fp8_scale(epi.sb, epi.hist, epi.fb));
  const float qs = epi.q8 ? fp8_scale(epi.q8_st, epi.hist, epi.q8_fmax) : 1.f;
  float amax = 0.f;
  float* sC = (float*)smem;
  constexpr int CH = QR / 8;
  if constexpr (EP == 1) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int m = p0 + prow + i * 16 + fr;
        const int n = q0 + qrow + j * 16 + fq * 4;
        if (m < P && n < Q) {
          const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2],
                              acc[i][j][3]};
          store4(epi, alpha, gi, m, n, v, qs, &amax);
        }
      }
  }
  if constexpr (EP == 2) {
    // register epilogue: lane quads finished and packed to bf16 into a bf16
    // image of the C tile (one pass), then whole 16-B row chunks out (and
    // the fp8 copy from the same bf16 values)
    constexpr int LDO = QR + 8;
    static_assert(PR * LDO * 2 <= 2 * SST, "bf16 C tile fits the ring");
    uint16_t* sO = (uint16_t*)smem;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int ml = prow + i * 16 + fr, nl = qrow + j * 16 + fq * 4;
        const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2],
                            acc[i][j][3]};
        uint2 o = make_uint2(0u, 0u);
        if (p0 + ml < P && q0 + nl < Q)
          o = pre4_8(epi, alpha, gi, p0 + ml, q0 + nl, v);
        *(uint2*)(sO + ml * LDO + nl) = o;
      }
    __syncthreads();
    for (int q = t; q < PR * CH; q += 256) {
      const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
      if (p0 + row >= P || q0 + c8 >= Q) continue;
      const uint4 ob = *(const uint4*)(sO + row * LDO + c8);
      const long long idx =
          (long long)(p0 + row) * epi.ldc + q0 + c8 + gi * epi.gcol;
      *(uint4*)(epi.c + idx) = ob;
      if (epi.q8) q8_out8(epi, idx, ob, qs, &amax);
    }
  }
#pragma unroll
  for (int e = 0; e < (EP != 0 ? 0 : 2); ++e) {
    if (e) __syncthreads();
    if ((w >> 1) == e) {    // the waves holding P rows e*HP .. +HP-1
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int rb = prow - e * HP + i * 16 + fq * 4;
          const int qc = qrow + j * 16 + fr;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) sC[(rb + rr) * LDC + qc] = acc[i][j][rr];
        }
    }
    __syncthreads();
    const int m0 = p0 + e * HP;
    for (int q = t; q < HP * CH; q += 256) {
      const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
      if (m0 + row >= P) continue;
      const float4* src = (const float4*)(sC + row * LDC + c8);
      float v[8];
      const float4 lo = src[0], hi = src[1];
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      store8(epi, alpha, gi, m0 + row, q0 + c8, v, qs, &amax);
    }
  }
  if (epi.q8) {
    amax = wave_max(amax);
    __syncthreads();
    float* red = (float*)smem;
    if (lane == 0) red[w] = amax;
    __syncthreads();
    if (t == 0) {
      float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      if (mx > 0.f)
        atomicMax((unsigned int*)(epi.q8_shard + (blockIdx.x & 31) * 32),
                  __float_as_uint(mx));
    }
  }
}

// convolutions on the T4 fp8 loop when the output channels per group fill
// 128-wide tiles (<= 1/8 wasted) - VGG's 128..512; hvk_fp8_variant 71
// keeps the 128-row loop (A/B runs)
inline bool want_t4_fp8(int N) {
  if (hvk_fp8_variant == 71) return false;
  if (N > 48 && N <= 64) return hvk_fp8_variant != 72;   // 256 x 64 tiles
  const int w = (N + 127) / 128 * 128 - N;
  return N >= 128 && w * 8 <= N;
}

template <class LP, int FA, int FB, int EP>
hipError_t go_t4_fp8_(const LP& lp, const Dense8& lq, const Epi8& e, int M,
                      int N, int K, int groups, hipStream_t s) {
  if (N <= 64) {
    const int tiles = (M + 255) / 256;
    hipLaunchKernelGGL((gemm_t4_fp8_kernel<LP, FA, FB, 256, 64, EP>),
                       dim3((unsigned)((long long)tiles * groups)), dim3(256),
                       0, s, lp, lq, e, M, N, K, 1, tiles, 1);
    return launch_status(s);
  }
  const int tiles_q = (N + 127) / 128;
  const int tiles = (M + 191) / 192 * tiles_q;
  const int gm = tiles_q >= 8 ? 8 : 1;
  hipLaunchKernelGGL((gemm_t4_fp8_kernel<LP, FA, FB, 192, 128, EP>),
                     dim3((unsigned)((long long)tiles * groups)), dim3(256), 0,
                     s, lp, lq, e, M, N, K, tiles_q, tiles, gm);
  return launch_status(s);
}

// the direct epilogue is opt-in (hvk_fp8_variant 74): measured slower than
// the LDS-staged one (VGG b512 conv2_2 forward 1241 -> 868 TF, conv1_2
// 640 -> 581; the 8-B lane quads leave 32-B pieces of each output row per
// store instruction)
template <class LP, int FA, int FB>
hipError_t go_t4_fp8(const LP& lp, const Dense8& lq, const Epi8& e, int M,
                     int N, int K, int groups, hipStream_t s) {
  if (hvk_fp8_variant == 74 && store4_ok(e))
    return go_t4_fp8_<LP, FA, FB, 1>(lp, lq, e, M, N, K, groups, s);
  // the register epilogue with a bf16 C image: opt-in (hvk_fp8_variant 73),
  // as in the bf16 loop, where it measured slower than the f32 staging
  if (hvk_fp8_variant == 73 && regepi_ok(e))
    return go_t4_fp8_<LP, FA, FB, 2>(lp, lq, e, M, N, K, groups, s);
  return go_t4_fp8_<LP, FA, FB, 0>(lp, lq, e, M, N, K, groups, s);
}

// ---------------------------------------------------------------------------
// 256 x 256 fp8 tile on the bf16 four-phase ping-pong schedule (gemm_pp.h
// gemm_pp256_kernel: 1.42 PF bf16 at 8192^3).  A K tile of 128 fp8 bytes is
// byte-for-byte the bf16 loop's 64-element tile (128-B rows, chunk c at
// c ^ (row & 7), 1-KiB LDS-DMA pieces of 8 rows), and a 16x16x128 f8f6f4
// MFMA (32 cycles) consumes the 32 B a lane holds for both halves of the
// bf16 K tile: per K tile a wave issues the same 24 fragment reads and 8
// DMA pieces against 32 MFMAs that each do twice the bf16 work - the same
// schedule at the fp8 rate.  Two groups of four waves, group 1 one barrier
// behind; quadrant phases q0..q3 read A0 + B0 / B1 / A1 / nothing, A(t+1)
// is DMAed in q0 / q1 into the stage tile t-1 left, B(t+2) in q2 / q3 into
// tile t's stage once its B reads are retired, one vmcnt(4) per tile (the
// slot-numbered RAW / WAR argument of gemm_pp.h holds unchanged).
struct PP8Op {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t v[4];
  int kc;
  __device__ __forceinline__ void init(const Dense8& l, int r0, int w,
                                       int lane) {
    rs = dma_rsrc(l.p);
    kc = 16 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = l.row_voff(r0 + 8 * (w * 4 + i) + (lane >> 3));
  }
  __device__ __forceinline__ void issue(const Dense8& l, int k0, uint8_t* s,
                                        int w, int i0, int n) {
    const bool kin = k0 + kc < l.K;
    const uint32_t kb = (uint32_t)(k0 + kc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i >= i0 && i < i0 + n)
        dma16(rs, s + (w * 4 + i) * 1024, kin ? v[i] + kb : kBufOOB);
  }
};

// the implicit-GEMM conv operand (ConvFwdA8 / ConvDgradA8) of the same
// loop: pieces as PP8Op, addresses from the row's DRow and the K tile's
// DTap (fast conv addressing, conv_geom.h)
template <class L>
struct PP8OpC {
  DRow fa[4];
  int kc;
  __device__ __forceinline__ void init(const L& l, int r0, int w, int lane) {
    kc = 16 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = l.drow(r0 + 8 * (w * 4 + i) + (lane >> 3));
  }
  __device__ __forceinline__ void issue(const L& l, int k0, uint8_t* s, int w,
                                        int i0, int n) {
    const DTap tp = l.dtap(k0 + kc);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i >= i0 && i < i0 + n)
        __builtin_amdgcn_global_load_lds(
            (const void*)l.dsrc(fa[i], tp),
            (__attribute__((address_space(3))) void*)(s + (w * 4 + i) * 1024),
            16, 0, 0);
  }
};

// LP: Dense8 (dense GEMMs) or a conv A loader (groups: blockIdx over
// tiles x groups)
template <class LP, int FA, int FB>
__global__ void __launch_bounds__(512, 1)
gemm_pp256_fp8_kernel(LP lp, Dense8 lq, Epi8 epi, int P, int Q, int K,
                      int tiles_q, int tiles, int gm) {
  constexpr int TB = 256 * BK;           // bytes per operand stage
  constexpr int SST = 2 * TB;            // A + B
  constexpr int LDC = 256 + 4;
  static_assert(64 * LDC * 4 <= 2 * SST, "epilogue pass fits");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * SST];
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gi = wgid / tiles;
  int tp, tq;
  if (gm > 1) {
    const int tiles_p = tiles / tiles_q;
    const int g = tile / (gm * tiles_q);
    const int p0g = g * gm;
    const int gh = min(tiles_p - p0g, gm);
    const int r = tile - g * gm * tiles_q;
    tp = p0g + r % gh;
    tq = r / gh;
  } else {
    tp = tile / tiles_q;
    tq = tile - tp * tiles_q;
  }
  if constexpr (!std::is_same<LP, Dense8>::value) lp.group(gi);
  lq.group(gi);
  const int p0 = tp * 256, q0 = tq * 256;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int grp = w >> 2;
  const int prow = grp * 128, qrow = (w & 3) * 64;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typename std::conditional<std::is_same<LP, Dense8>::value, PP8Op,
                            PP8OpC<LP>>::type op;
  PP8Op oq;
  op.init(lp, p0, w, lane);
  oq.init(lq, q0, w, lane);
  // 32 bytes of row (rowbase + fr): chunks fq, fq + 4 at c ^ (row & 7)
  // (the k assignment the 128-row loop uses; conflict-free reads)
  auto frag = [&](const uint8_t* sb, int rowbase) -> i32x8 {
    const int row = rowbase + fr;
    const int sw = row & 7;
    const uint8_t* base = sb + row * BK;
    const uint4 lo = *(const uint4*)(base + ((fq ^ sw) << 4));
    const uint4 hi = *(const uint4*)(base + (((fq + 4) ^ sw) << 4));
    i32x8 v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  const int nk = (K + BK - 1) / BK;
  uint8_t* st0 = smem;
  uint8_t* st1 = smem + SST;
  op.issue(lp, 0, st0, w, 0, 4);
  oq.issue(lq, 0, st0 + TB, w, 0, 4);
  if (nk > 1) {
    oq.issue(lq, BK, st1 + TB, w, 0, 4);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger group 1
  asm volatile("" ::: "memory");

  i32x8 af[4], b0[2], b1[2];
  auto mfma = [&](int abase, i32x8 (&bf)[2], int bbase) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[abase + i][bbase + j] =
            __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                af[i], bf[j], acc[abase + i][bbase + j], FA, FB, 0, 127, 0,
                127);
    __builtin_amdgcn_s_setprio(0);
  };
  auto slot_end = [&]() {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int kt = 0; kt < nk; ++kt) {
    const uint8_t* sP = (kt & 1) ? st1 : st0;
    const uint8_t* sQ = sP + TB;
    uint8_t* nxt = (kt & 1) ? st0 : st1;
    uint8_t* cur = (kt & 1) ? st1 : st0;
    const bool pa = kt + 1 < nk, pb = kt + 2 < nk;
    const int ka = (kt + 1) * BK, kb = (kt + 2) * BK;
    // q0 MEM: A0, B0; A(t+1) pieces 0, 1
#pragma unroll
    for (int j = 0; j < 2; ++j) b0[j] = frag(sQ, qrow + j * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(sP, prow + i * 16);
    if (pa) op.issue(lp, ka, nxt, w, 0, 2);
    slot_end();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma(0, b0, 0);
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // q1 MEM: B1; A(t+1) pieces 2, 3
#pragma unroll
    for (int j = 0; j < 2; ++j) b1[j] = frag(sQ, qrow + 32 + j * 16);
    if (pa) op.issue(lp, ka, nxt, w, 2, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    slot_end();
    mfma(0, b1, 2);
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // q2 MEM: A1; B(t+2) pieces 0, 1
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(sP, prow + 64 + i * 16);
    if (pb) oq.issue(lq, kb, cur + TB, w, 0, 2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    slot_end();
    mfma(4, b1, 2);
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // q3 MEM: B(t+2) pieces 2, 3; wait for tile t+1
    if (pb) {
      oq.issue(lq, kb, cur + TB, w, 2, 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    slot_end();
    mfma(4, b0, 0);
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // group 1's last slot
  asm volatile("" ::: "memory");

  const float alpha = 1.f / (fp8_scale(epi.sa, epi.hist, epi.fa) *
                             fp8_scale(epi.sb, epi.hist, epi.fb));
  const float qs = epi.q8 ? fp8_scale(epi.q8_st, epi.hist, epi.q8_fmax) : 1.f;
  float amax = 0.f;
  float* sC = (float*)smem;
  constexpr int CH = 256 / 8;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __syncthreads();
    if (grp == (e >> 1)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rb = i * 16 + fq * 4;
          const int qc = qrow + j * 16 + fr;
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            sC[(rb + rr) * LDC + qc] = acc[(e & 1) * 4 + i][j][rr];
        }
    }
    __syncthreads();
    const int m0 = p0 + e * 64;
    for (int q = t; q < 64 * CH; q += 512) {
      const int row = q / CH, c8 = (q % CH) * 8;
      if (m0 + row >= P) continue;
      const float4* src = (const float4*)(sC + row * LDC + c8);
      float v[8];
      const float4 lo = src[0], hi = src[1];
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      store8(epi, alpha, gi, m0 + row, q0 + c8, v, qs, &amax);
    }
  }
  if (epi.q8) {
    amax = wave_max(amax);
    __syncthreads();
    float* red = (float*)smem;
    if (lane == 0) red[w] = amax;
    __syncthreads();
    if (t == 0) {
      float mx = 0.f;
      for (int i = 0; i < 8; ++i) mx = fmaxf(mx, red[i]);
      if (mx > 0.f)
        atomicMax((unsigned int*)(epi.q8_shard + (blockIdx.x & 31) * 32),
                  __float_as_uint(mx));
    }
  }
}

// the 256 x 256 loop for dense fp8 GEMMs with at least one tile per CU
// (hvk_gemm_variant 70 keeps the 128-row loop: A/B runs)
inline bool want_pp256_fp8(const Dense8& la, const Dense8& lb, int M, int N) {
  if (hvk_fp8_variant == 70) return false;
  if (!la.buf_ok() || !lb.buf_ok()) return false;
  const long long t = (long long)((M + 255) / 256) * ((N + 255) / 256);
  const int wn = (N + 255) / 256 * 256 - N;
  return t >= 256 && wn * 8 <= N;
}

template <class LA, int FA, int FB>
hipError_t go_pp256_fp8(const LA& la, const Dense8& lb, const Epi8& e, int M,
                        int N, int K, int groups, hipStream_t s) {
  const int tiles_q = (N + 255) / 256;
  const int tiles = (M + 255) / 256 * tiles_q;
  const int gm = tiles_q >= 8 ? 8 : 1;
  hipLaunchKernelGGL((gemm_pp256_fp8_kernel<LA, FA, FB>),
                     dim3((unsigned)((long long)tiles * groups)), dim3(512), 0,
                     s, la, lb, e, M, N, K, tiles_q, tiles, gm);
  return launch_status(s);
}

// fp8 convolutions with >= 256 outputs per group (VGG conv3-5 forward and
// backward-data) on the 256 x 256 loop where it fills the CUs (<= 1/8 of the
// column tile wasted, >= one tile per CU); default settings only,
// hvk_fp8_variant 75 forces it (tests)
inline bool want_pp256_fp8_conv(const Dense8& lb, int M, int N, int groups) {
  if (!lb.buf_ok()) return false;
  const int wn = (N + 255) / 256 * 256 - N;
  if (N < 256 || wn * 8 > N) return false;
  if (hvk_fp8_variant == 75) return true;
  if (hvk_fp8_variant >= 0) return false;
  return (long long)((M + 255) / 256) * ((N + 255) / 256) * groups >= 256;
}

inline bool use_bn64(int N) {
  int w128 = (N + 127) / 128 * 128 - N;
  int w64 = (N + 63) / 64 * 64 - N;
  return w64 < w128 && w128 * 8 > N;
}

template <class LA, class LB, int FA, int FB>
hipError_t launch8(const LA& la, const LB& lb, const Epi8& e, int M, int N,
                   int K, int groups, hipStream_t s) {
  if constexpr (std::is_same<LA, Dense8>::value &&
                std::is_same<LB, Dense8>::value) {
    if (groups == 1 && want_pp256_fp8(la, lb, M, N))
      return go_pp256_fp8<Dense8, FA, FB>(la, lb, e, M, N, K, 1, s);
  }
  if constexpr ((std::is_same<LA, ConvFwdA8>::value ||
                 std::is_same<LA, ConvDgradA8>::value) &&
                std::is_same<LB, Dense8>::value) {
    if (want_pp256_fp8_conv(lb, M, N, groups))
      return go_pp256_fp8<LA, FA, FB>(la, lb, e, M, N, K, groups, s);
    // the 256 x 64 tiles for forward convolutions only: VGG b512 conv1_2
    // backward-data (with the derivative of the layer below in the
    // epilogue) took 3.97 ms on them against 3.55 ms on the 128-row loop,
    // the forward 3.02 against 3.19 (profiles/r4/vgg16_b512_fp8_step_r4h.md)
    const bool t4_64_dgrad = std::is_same<LA, ConvDgradA8>::value && N <= 64 &&
                             hvk_fp8_variant != 75;
    if (want_t4_fp8(N) && !t4_64_dgrad)
      return go_t4_fp8<LA, FA, FB>(la, lb, e, M, N, K, groups, s);
  }
  const bool n64 = use_bn64(N);
  const int bn = n64 ? 64 : 128;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + bn - 1) / bn;
  const int tiles = tiles_m * tiles_n;
  dim3 grid((unsigned)((long long)tiles * groups));
  // 8-wave blocks (profiles/gemm_experiments_r2.md section 8)
  if (n64)
    hipLaunchKernelGGL((gemm_fp8_kernel<LA, LB, 64, FA, FB, true>), grid,
                       dim3(512), 0, s, la, lb, e, M, N, K, tiles_n, tiles);
  else
    hipLaunchKernelGGL((gemm_fp8_kernel<LA, LB, 128, FA, FB, true>), grid,
                       dim3(512), 0, s, la, lb, e, M, N, K, tiles_n, tiles);
  return launch_status(s);
}

// fmt: 0 = e4m3 (fp8), 1 = e5m2 (bf8) -> the f8f6f4 cbsz/blgp codes.  B is
// always a weight (e4m3); A is an activation (e4m3) or a gradient (e5m2).
template <class LA, class LB>
hipError_t dispatch8(int fa, int fb, const LA& la, const LB& lb,
                     const Epi8& e, int M, int N, int K, int groups,
                     hipStream_t s) {
  if (fb != 0) return hipErrorInvalidValue;
  if (fa == 0) return launch8<LA, LB, 0, 0>(la, lb, e, M, N, K, groups, s);
  return launch8<LA, LB, 1, 0>(la, lb, e, M, N, K, groups, s);
}

Epi8 make_epi8(void* c, int ldc, int M, int N, const float* bias, int act,
               const void* aux, int ld_aux, int aux_act, const float* sa,
               const float* sb, int hist, float fa, float fb) {
  Epi8 e;
  e.c = (uint16_t*)c; e.ldc = ldc; e.M = M; e.N = N;
  e.grow_unused = 0; e.gcol = 0; e.bias = bias; e.act = act;
  e.aux = (const uint16_t*)aux; e.ld_aux = ld_aux; e.aux_act = aux_act;
  e.sa = sa; e.sb = sb; e.hist = hist; e.fa = fa; e.fb = fb;
  e.q8 = nullptr; e.q8_st = nullptr; e.q8_shard = nullptr; e.q8_fmax = 1.f;
  e.q8_fmt = 0;
  return e;
}

// -------------------------------------------------------------- quantizers

// Units of 8 elements (one 16-B bf16 load or two float4 loads -> one 8-B
// fp8 store), lanes on consecutive units so every load is fully coalesced;
// each thread keeps UNR units in flight per iteration.  amax of |x|
// (unscaled) goes to st[hist] with an integer atomicMax on the float bits
// (non-negative floats order like their bit patterns).
template <bool F32>
__device__ __forceinline__ void load8(const void* x, long long u, float* v) {
  if constexpr (F32) {
    const float4* p = (const float4*)x + u * 2;
    float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    uint4 w = ((const uint4*)x)[u];
    const uint16_t* h = (const uint16_t*)&w;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = bf2f(h[q]);
  }
}

// amax of the whole workgroup (256 threads) -> one atomicMax per workgroup:
// thousands of same-address atomics serialise in L2 (~12 ns each)
__device__ __forceinline__ void record_amax(float amax, float* slot) {
  __shared__ float red[4];
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (m > 0.f) atomicMax((unsigned int*)slot, __float_as_uint(m));
  }
}

template <bool F32>
__global__ void fp8_quant_kernel(const void* x, long long n, uint8_t* out,
                                 int fmt, float* st, int hist, float fmax_eff,
                                 float lim, int record) {
  constexpr int UNR = 4;
  const float scale = fp8_scale(st, hist, fmax_eff);
  float amax = 0.f;
  const long long nu = n / 8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long u0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       u0 < nu; u0 += stride * UNR) {
    float v[UNR][8];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const long long u = u0 + k * stride;
      if (u < nu) load8<F32>(x, u, v[k]);
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const long long u = u0 + k * stride;
      if (u >= nu) break;
      uint2 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(v[k][q]));
      o.x = pack4_fp8(sat(v[k][0] * scale, lim), sat(v[k][1] * scale, lim),
                      sat(v[k][2] * scale, lim), sat(v[k][3] * scale, lim), fmt);
      o.y = pack4_fp8(sat(v[k][4] * scale, lim), sat(v[k][5] * scale, lim),
                      sat(v[k][6] * scale, lim), sat(v[k][7] * scale, lim), fmt);
      ((uint2*)out)[u] = o;
    }
  }
  // scalar tail (n % 8)
  const long long tail0 = nu * 8;
  if (blockIdx.x == 0 && threadIdx.x < n - tail0) {
    const long long e = tail0 + threadIdx.x;
    float v = F32 ? ((const float*)x)[e] : bf2f(((const uint16_t*)x)[e]);
    amax = fmaxf(amax, fabsf(v));
    out[e] = (uint8_t)(pack4_fp8(sat(v * scale, lim), 0.f, 0.f, 0.f, fmt) & 0xFF);
  }
  if (record) record_amax(amax, st + hist);
}

template <bool F32>
__global__ void fp8_amax_kernel(const void* x, long long n, float* st,
                                int hist) {
  float amax = 0.f;
  const long long nu = n / 8;
  for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nu;
       u += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8<F32>(x, u, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(v[q]));
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nu * 8) {
    const long long e = nu * 8 + threadIdx.x;
    amax = fmaxf(amax, fabsf(F32 ? ((const float*)x)[e]
                                 : bf2f(((const uint16_t*)x)[e])));
  }
  record_amax(amax, st + hist);
}

// history[idx] = current amax (or every slot when fill), current = 0; one
// thread per scaler of a [count][hist + 1] state block
// step (optional): the history slot is step % hist read from device memory
// (graph-safe roll; the registry advances the counter after the launch)
__global__ void fp8_roll_kernel(float* states, int count, int hist, int idx,
                                int fill, const int* step, float* shards) {
  if (step) idx = __builtin_amdgcn_readfirstlane(step[0]) % hist;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  float* st = states + (long long)s * (hist + 1);
  float cur = st[hist];
  if (shards) {   // amaxes recorded by fused-quantising epilogues
    float* sh = shards + (long long)s * 1024;
    for (int i = 0; i < 32; ++i) {
      cur = fmaxf(cur, sh[i * 32]);
      sh[i * 32] = 0.f;
    }
  }
  if (fill) {
    for (int i = 0; i < hist; ++i) st[i] = cur;
  } else if (cur > 0.f) {
    st[idx] = cur;
  }
  st[hist] = 0.f;
}

// at most 1024 workgroups (4 per CU): the grid-stride loops keep enough
// bytes in flight, and the amax atomics stay few
inline int grid_for(long long work, int per_block) {
  long long b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > 1024) b = 1024;
  return (int)b;
}

}  // namespace

// out (fp8, n bytes) = sat(x * scale(st)); st[hist] = max(st[hist], amax|x|)
HVK_API int hvk_fp8_quant(const void* x, int x_f32, long long n, void* out,
                          int fmt, float* st, int hist, float fmax_eff,
                          int record, hipStream_t s) {
  if (((uintptr_t)x & 15) || ((uintptr_t)out & 15)) return -3;
  const float lim = fmt == 0 ? 448.f : 57344.f;
  const dim3 grid(grid_for(n / 32 + 1, 256));
  if (x_f32)
    hipLaunchKernelGGL(fp8_quant_kernel<true>, grid, dim3(256), 0, s, x, n,
                       (uint8_t*)out, fmt, st, hist, fmax_eff, lim, record);
  else
    hipLaunchKernelGGL(fp8_quant_kernel<false>, grid, dim3(256), 0, s, x, n,
                       (uint8_t*)out, fmt, st, hist, fmax_eff, lim, record);
  return (int)launch_status(s);
}

HVK_API int hvk_fp8_amax(const void* x, int x_f32, long long n, float* st,
                         int hist, hipStream_t s) {
  if (((uintptr_t)x & 15)) return -3;
  const dim3 grid(grid_for(n / 8 + 1, 256));
  if (x_f32)
    hipLaunchKernelGGL(fp8_amax_kernel<true>, grid, dim3(256), 0, s, x, n, st,
                       hist);
  else
    hipLaunchKernelGGL(fp8_amax_kernel<false>, grid, dim3(256), 0, s, x, n,
                       st, hist);
  return (int)launch_status(s);
}

// shards (optional): [count][1024] f32, 32 amax shards per scaler 32 floats
// apart, folded into the current amax and cleared
HVK_API int hvk_fp8_roll(float* states, int count, int hist, int idx,
                         int fill, float* shards, hipStream_t s) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(fp8_roll_kernel, dim3((count + 63) / 64), dim3(64), 0, s,
                     states, count, hist, idx, fill, (const int*)nullptr,
                     shards);
  return (int)launch_status(s);
}

HVK_API int hvk_fp8_roll_dev(float* states, int count, int hist,
                             const void* step, float* shards, hipStream_t s) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(fp8_roll_kernel, dim3((count + 63) / 64), dim3(64), 0, s,
                     states, count, hist, 0, 0, (const int*)step, shards);
  return (int)launch_status(s);
}

// the fused quantisation of an fp8 conv's output (Epi8::q8); q8 == nullptr
// leaves it off
inline void set_q8(Epi8& e, void* q8, const float* st, float* shard,
                   float fmax, int fmt) {
  e.q8 = (uint8_t*)q8;
  e.q8_st = st;
  e.q8_shard = shard;
  e.q8_fmax = fmax;
  e.q8_fmt = fmt;
}

HVK_API void hvk_set_fp8_variant(int v) { hvk_fp8_variant = v; }

// C[M][N] (bf16) = act(A[M][K] . B[N][K]^T / (sA sB) + bias) * f'(aux)
HVK_API int hvk_gemm_fp8(int M, int N, int K, const void* A, int lda, int fa,
                         const void* B, int ldb, int fb, void* C, int ldc,
                         const float* bias, int act, const void* aux,
                         int ld_aux, int aux_act, const float* sa,
                         const float* sb, int hist, float fmax_a, float fmax_b,
                         hipStream_t s) {
  if ((K & 15) || (lda & 15) || (ldb & 15) || !al16(A) || !al16(B)) return -3;
  Dense8 la{(const uint8_t*)A, 0, M, K, lda};
  Dense8 lb{(const uint8_t*)B, 0, N, K, ldb};
  Epi8 e = make_epi8(C, ldc, M, N, bias, act, aux, ld_aux, aux_act, sa, sb,
                     hist, fmax_a, fmax_b);
  return (int)dispatch8(fa, fb, la, lb, e, M, N, K, 1, s);
}

// Y[n][oh][ow][oc] (bf16) = act(conv(X8, W8) / (sX sW) + bias)
// X8 NHWC fp8, W8 [OC][KH][KW][C/g] fp8; C/g, C and K multiples of 16
HVK_API int hvk_conv_fwd_fp8(const void* X, const void* Wt, const float* bias,
                             void* Y, int N, int H, int W, int C, int OC,
                             int KH, int KW, int sy, int sx, int pt, int pl,
                             int OH, int OW, int groups, int act, int fx,
                             int fw, const float* sxs, const float* sws,
                             int hist, float fmax_x, float fmax_w, void* q8,
                             const float* q8_st, float* q8_shard,
                             float q8_fmax, int q8_fmt, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  const int M = N * OH * OW, K = KH * KW * g.Cg;
  if ((g.Cg & 15) || (C & 15) || !al16(X) || !al16(Wt) || KH > 32 ||
      KW > 32)
    return -3;
  ConvFwdA8 la{(const uint8_t*)X, g, M, K, 0};
  Dense8 lb{(const uint8_t*)Wt, (long long)g.OCg * K, g.OCg, K, K};
  Epi8 e = make_epi8(Y, OC, M, g.OCg, bias, act, nullptr, 0, 0, sxs, sws,
                     hist, fmax_x, fmax_w);
  e.gcol = g.OCg;
  if (q8 && (((uintptr_t)q8) & 7)) return -3;
  set_q8(e, q8, q8_st, q8_shard, q8_fmax, q8_fmt);
  return (int)dispatch8(fx, fw, la, lb, e, M, g.OCg, K, groups, s);
}

// dX (bf16) = conv^T(dY8, Wt8) / (sdY sW) [* f'(aux)]; Wt8 is the weight
// permuted to [g][c][kh][kw][oc] (dense K-major per group)
HVK_API int hvk_conv_dgrad_fp8(const void* dY, const void* Wt, void* dX,
                               int N, int H, int W, int C, int OC, int KH,
                               int KW, int sy, int sx, int pt, int pl, int OH,
                               int OW, int groups, const void* aux,
                               int aux_act, int fdy, int fw, const float* sds,
                               const float* sws, int hist, float fmax_dy,
                               float fmax_w, void* q8, const float* q8_st,
                               float* q8_shard, float q8_fmax, int q8_fmt,
                               hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  const int M = N * H * W, K = KH * KW * g.OCg;
  if ((g.OCg & 15) || (OC & 15) || !al16(dY) || !al16(Wt)) return -3;
  ConvDgradA8 la{(const uint8_t*)dY, g, M, K, 0};
  Dense8 lb{(const uint8_t*)Wt, (long long)K * g.Cg, g.Cg, K, K};
  Epi8 e = make_epi8(dX, C, M, g.Cg, nullptr, 0, aux, C, aux_act, sds, sws,
                     hist, fmax_dy, fmax_w);
  e.gcol = g.Cg;
  if (q8 && (((uintptr_t)q8) & 7)) return -3;
  set_q8(e, q8, q8_st, q8_shard, q8_fmax, q8_fmt);
  if (sy != 1 || sx != 1 || KH > 32 || KW > 32) {
    ConvDgradA8Str ls;
    static_cast<ConvDgradA8&>(ls) = la;
    return (int)dispatch8(fdy, fw, ls, lb, e, M, g.Cg, K, groups, s);
  }
  return (int)dispatch8(fdy, fw, la, lb, e, M, g.Cg, K, groups, s);
}
