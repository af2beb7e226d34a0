// gemm_pp.h - ping-pong main loop for large bf16 GEMM / implicit-GEMM
// convolution tiles (LDS-DMA operands).  Included by gemm_core.h inside its
// anonymous namespace, after the loaders and Epi.
//
// Why a second main loop: the 128 x BN / 2-barriers-per-K-tile loop of
// gemm_kernel is bound by moving its operands (profiles/r3_experiments.md §10:
// with the LDS-DMA removed after the first K tile the 8192^3 GEMM runs 2x
// faster; halving its MFMAs takes 2 % off).  This loop moves 0.75x the bytes
// per FLOP (256 x 128 tile) and keeps the DMA off the MFMA critical path:
//
//   * 8 waves = two groups of 4 (one wave of each group per SIMD).  Group g
//     owns tile rows g*128 .. +128 of the 256-row tile; inside a group the
//     waves are 2 x 2, each 64 x 64 (4 x 4 MFMA 16x16x32 accumulators).
//   * a K tile (BK = 64) is two phases; a phase = MEM slot (ds_read the
//     fragments for this phase, issue this phase's LDS-DMA pieces, counted
//     waits) then MFMA slot (16 MFMAs), each slot closed by s_barrier.
//   * group 1 runs one barrier behind group 0, so on every SIMD one wave is
//     in its MFMA slot while the other is in its MEM slot (ping-pong): LDS
//     read latency and DMA issue hide under the other group's MFMAs.
//   * 3-stage LDS ring (3 x 48 KiB): during K tile t the waves DMA tile t+2
//     (the 256-row operand in phase 0, the 128-row one in phase 1); tile t+1
//     is waited for with vmcnt(6) in phase 1 (tile t+2's six pieces stay in
//     flight), so every piece has 4-6 slots to land.  One workgroup per CU.
//
// Hazards, by barrier-delimited slot number (group g, phase P = 2t + ph: MEM
// slot 2P + g, MFMA slot 2P + g + 1):
//   RAW  tile t+1 is waited for in slots 4t+2 (g0) / 4t+3 (g1), both before
//        the barrier that ends them; its first reads are in slots 4t+4 / 4t+5.
//   WAR  stage (t+2)%3 held tile t-1, last read in slot 4t-1 (g1, phase 1,
//        lgkmcnt(0) before that slot's barrier); its first DMA is issued in
//        slot 4t (g0).
//
// Operands: the LDS images and DMA addressing of gemm_kernel - K-major
// [rows][64 k] (16-B chunk c of row r at c ^ (r & 7), ds_read_b128
// fragments) or MN-major [64 k][128 cols] images (32-B block b of k-row k at
// b ^ hk(k), ds_read_b64_tr_b16 fragments), written lane-linear by the DMA
// from pre-permuted source offsets.  Every loader keeps its own addressing.
//
// Measured against gemm_kernel (tools/bench_gemm_ab.py, profiles/
// r3_experiments.md §12): +8..14 % on the large dense NT / NN GEMMs; slower on
// the implicit-GEMM convolutions and short-K / TN weight gradients, which keep
// gemm_kernel (one workgroup per CU cannot overlap one tile's prologue and
// epilogue with another's main loop).

constexpr int PP_BM = 256, PP_BN = 128, PP_NST = 3;
constexpr int PP_SA = PP_BM * BK, PP_SB = PP_BN * BK, PP_SST = PP_SA + PP_SB;
constexpr int PP_LDC = PP_BN + 4;      // staged epilogue row pitch (floats)
constexpr int PP_SMEM_BYTES = PP_NST * PP_SST * 2;
static_assert(PP_BM * PP_LDC * 4 <= PP_SMEM_BYTES,
              "epilogue staging fits the ring");

// the operands the ping-pong loop takes (measured, profiles/r3_experiments.md
// §12): dense K-major A (DenseK) against dense K-major or MN-major B (NT / NN
// GEMMs).  The implicit-GEMM convolutions and the MN-major-A (TN) weight
// gradients ran 2-50 % slower on it than on gemm_kernel's two workgroups per
// CU and stay there.
template <class L, bool KM, bool ISP>
constexpr bool pp_loader_ok() {
  if constexpr (ISP) return KM && std::is_same<L, DenseK>::value;
  else return std::is_same<L, DenseK>::value || std::is_same<L, DenseMN>::value;
}

// One operand's DMA slots.  ROWS (256 / 128) x 64 k of bf16 = ROWS / 64
// pieces of 1 KiB per wave.  K-major slot I: rows 8I .. 8I+7, all 8 chunks;
// MN-major slot I: image I / 16 (128 columns each), k-rows 4 (I % 16) .. +3.
// K-major implicit-GEMM conv operands (ConvFwdA / ConvDgradA, kFast): the
// row's pixel and tap masks once (DRow), the lane's tap once per K tile
// (DTap), as in the T4 loop
// The MN-major conv weight-gradient operand (ConvWgradB, kFast: the im2col
// column's tap fixed, a running pixel advanced by BK per K tile, pointer
// LDS-DMA as in the T4 loop): MNFAST.  Its pieces must be issued once per K
// tile, in K order (the 256 x 256 loop issues each piece exactly once).
template <class L, bool KM, int ROWS>
struct PPOp {
  static constexpr int NS = ROWS / 64;
  static constexpr bool FAST = KM && L::kFast;
  static constexpr bool MNFAST = !KM && L::kFast;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t v[NS];
  int kr[NS];
  int kc;
  DRow fa[FAST ? NS : 1];
  typename DColOf<L, MNFAST>::type fb[MNFAST ? NS : 1];
  __device__ __forceinline__ void init(const L& l, int r0, int w, int lane,
                                       int kbeg = 0) {
    if constexpr (L::kBuf) rs = dma_rsrc(l.dbase());
    kc = 8 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int I = w * NS + i;
      if constexpr (FAST) {
        fa[i] = l.drow(r0 + 8 * I + (lane >> 3));
      } else if constexpr (KM) {
        v[i] = l.row_voff(r0 + 8 * I + (lane >> 3));
      } else {
        const int Ii = I & 15, h = I >> 4;
        const int hkv = ((lane >> 4) & 3) | (((Ii >> 1) & 1) << 2);
        const int c = ((((lane & 15) >> 1) ^ hkv) << 1) | (lane & 1);
        kr[i] = 4 * Ii + (lane >> 4);
        if constexpr (MNFAST)
          fb[i] = l.dcol(r0 + h * 128 + 8 * c, kbeg + kr[i], false);
        else
          v[i] = l.col_voff(r0 + h * 128 + 8 * c, kr[i]);
      }
    }
  }
  __device__ __forceinline__ static uint16_t* dst(uint16_t* s, int I) {
    if constexpr (KM) return s + I * 512;
    else return s + (I >> 4) * (64 * 128) + (I & 15) * 512;
  }
  // pieces [i0, i0 + n) of this wave only (the 256 x 256 loop issues an
  // operand's four pieces over two phases)
  __device__ __forceinline__ void issue_part(const L& l, int k0, uint16_t* s,
                                             int w, int i0, int n) {
    if constexpr (FAST) {
      const DTap tp = l.dtap(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if (i >= i0 && i < i0 + n)
          dma16(rs, dst(s, w * NS + i), l.dvoff(fa[i], tp));
    } else if constexpr (KM) {
      const bool kin = k0 + kc < l.K;
      const uint32_t kbyte = 2u * (uint32_t)(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if (i >= i0 && i < i0 + n)
          dma16(rs, dst(s, w * NS + i), kin ? v[i] + kbyte : kBufOOB);
    } else if constexpr (MNFAST) {
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if (i >= i0 && i < i0 + n) {
          __builtin_amdgcn_global_load_lds(
              (const void*)l.dsrc(fb[i]),
              (__attribute__((address_space(3))) void*)dst(s, w * NS + i), 16,
              0, 0);
          l.dnext_by(fb[i], BK);
        }
    } else {
      const uint32_t kadv = (uint32_t)k0 * (uint32_t)l.ld * 2u;
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if (i >= i0 && i < i0 + n)
          dma16(rs, dst(s, w * NS + i),
                k0 + kr[i] < l.K ? v[i] + kadv : kBufOOB);
    }
  }
  __device__ __forceinline__ void issue(const L& l, int k0, uint16_t* s, int w) {
    if constexpr (MNFAST) {
      issue_part(l, k0, s, w, 0, NS);
    } else if constexpr (FAST) {
      const DTap tp = l.dtap(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, dst(s, w * NS + i), l.dvoff(fa[i], tp));
    } else if constexpr (KM) {
      const bool kin = k0 + kc < l.K;
      const uint32_t kbyte = 2u * (uint32_t)(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, dst(s, w * NS + i), kin ? v[i] + kbyte : kBufOOB);
    } else {
      const uint32_t kadv = (uint32_t)k0 * (uint32_t)l.ld * 2u;
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, dst(s, w * NS + i), k0 + kr[i] < l.K ? v[i] + kadv : kBufOOB);
    }
  }
};

// fragment of a 16-row MFMA tile at `row` (16-row aligned), 32-deep half ks
template <bool KM>
__device__ __forceinline__ bf16x8 pp_frag(const uint16_t* s, int row, int ks,
                                          int fr, int fq) {
  if constexpr (KM) {
    const int r = row + fr;
    const int c = ks * 4 + fq;
    return *(const bf16x8*)(s + r * 64 + ((c ^ (r & 7)) << 3));
  } else {
    const uint16_t* im = s + (row >> 7) * (64 * 128);
    const int b = (row & 127) >> 4;
    const int trq = fr >> 2, trp = fr & 3;
    const int k = ks * 32 + fq * 8 + trq;
    const uint16_t* p0 = im + k * 128 + ((b ^ hk(k)) << 4) + trp * 4;
    const uint16_t* p1 = im + (k + 4) * 128 + ((b ^ hk(k + 4)) << 4) + trp * 4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

// LP / PK: the 256-row operand (rows P) and whether it is K-major; LQ / QK
// the 128-row one (rows Q): P x Q = M x N.
// ABL (diagnostic builds, hvk_gemm_variant 31; wrong results by design): 1 =
// no DMA after the prologue (the loop's MFMA / LDS / barrier cost alone)
template <class LP, bool PK, class LQ, bool QK, int ABL = 0>
__global__ void __launch_bounds__(512, 1)
gemm_pp_kernel(LP lp, LQ lq, Epi epi, int P, int Q, int K, int k_split,
               int tiles_q, int tiles, int splits, int gm) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[PP_SMEM_BYTES / 2];
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gs = wgid / tiles;
  const int gi = gs / splits;
  int tp, tq;
  if (gm > 1) {  // grouped tile order, as in gemm_kernel
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
  const int kbeg = (gs - gi * splits) * k_split;
  const int kend = min(K, kbeg + k_split);
  if (kbeg >= kend) return;
  lp.group(gi);
  lq.group(gi);
  const int p0 = tp * PP_BM, q0 = tq * PP_BN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int grp = w >> 2;
  const int prow = grp * 128 + ((w >> 1) & 1) * 64;  // wave's first P row
  const int qrow = (w & 1) * 64;                     // wave's first Q row
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  PPOp<LP, PK, PP_BM> op;
  PPOp<LQ, QK, PP_BN> oq;
  op.init(lp, p0, w, lane);
  oq.init(lq, q0, w, lane);
  constexpr int NIP = PPOp<LP, PK, PP_BM>::NS;
  constexpr int NIQ = PPOp<LQ, QK, PP_BN>::NS;
  static_assert(NIP + NIQ == 6, "vmcnt counts below assume 6 pieces per tile");

  const int nk = (kend - kbeg + BK - 1) / BK;
  // prologue: tiles 0 and 1 in flight, wait for tile 0
  op.issue(lp, kbeg, smem, w);
  oq.issue(lq, kbeg, smem + PP_SA, w);
  if (nk > 1) {
    op.issue(lp, kbeg + BK, smem + PP_SST, w);
    oq.issue(lq, kbeg + BK, smem + PP_SST + PP_SA, w);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one slot
  asm volatile("" ::: "memory");

  bf16x8 af[2][2], bfv[4][2];
  int scur = 0, spre = 2;  // stage of tile t, of tile t + 2
  for (int kt = 0; kt < nk; ++kt) {
    const uint16_t* sP = smem + scur * PP_SST;
    const uint16_t* sQ = sP + PP_SA;
    uint16_t* dP = smem + spre * PP_SST;
    const bool pre = kt + 2 < nk;
    const int kpre = kbeg + (kt + 2) * BK;
    // ---- phase 0, MEM: P rows 0..31 of the wave, all of its Q rows
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfv[j][ks] = pp_frag<QK>(sQ, qrow + j * 16, ks, fr, fq);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i][ks] = pp_frag<PK>(sP, prow + i * 16, ks, fr, fq);
    }
    if (pre && ABL != 1) op.issue(lp, kpre, dP, w);
    // no wait here: the fragment reads retire across the barrier (the MFMA
    // slot waits for them); tile t's stage is not restaged before tile t+1's
    // phase 0, and its last reads (phase 1) are retired before a barrier
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 0, MFMA
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i][ks], bfv[j][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 1, MEM: P rows 32..63; tile t + 2's Q; wait for tile t + 1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i][ks] = pp_frag<PK>(sP, prow + 32 + i * 16, ks, fr, fq);
    if (pre && ABL != 1) {
      oq.issue(lq, kpre, dP + PP_SA, w);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1, MFMA
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[2 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i][ks], bfv[j][ks], acc[2 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    scur = scur == 2 ? 0 : scur + 1;
    spre = spre == 2 ? 0 : spre + 1;
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // group 1's last slot
  asm volatile("" ::: "memory");

  // accumulator (i, j)[rr] is tile element (P row prow + 16i + 4fq + rr,
  // Q row qrow + 16j + fr)
  // stage the f32 tile through LDS (the ring is drained: every DMA waited
  // for, every fragment read retired before the last barrier), then
  // row-contiguous 16-B stores
  float* sC = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pb = prow + i * 16 + fq * 4;
      const int qc = qrow + j * 16 + fr;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        sC[(pb + rr) * PP_LDC + qc] = acc[i][j][rr];
      }
    }
  __syncthreads();
  constexpr int ROWS = PP_BM, LD = PP_LDC;
  const int m0 = p0, n0 = q0;
  if (epi.atomic) {
    // split-K partial sums: f32 atomics, a wave adding 64 consecutive
    // columns of one row per instruction (256 contiguous bytes: the full
    // atomic rate; 16 x 4 accumulator fragments straight from registers hit
    // 16 rows per instruction)
    constexpr int COLS = PP_BN;
    constexpr int RSTEP = 512 / COLS;
    const int c = t % COLS;
    for (int row = t / COLS; row < ROWS; row += RSTEP)
      epi.store(gi, m0 + row, n0 + c, sC[row * LD + c]);
    return;
  }
  constexpr int CH = PP_BN / 8;
  const bool fast = epi.fast_ok();
  for (int q = t; q < ROWS * CH; q += 512) {
    const int row = q / CH, c8 = (q % CH) * 8;
    if (m0 + row >= epi.M) continue;
    const float4* src = (const float4*)(sC + row * LD + c8);
    float v[8];
    const float4 lo = src[0], hi = src[1];
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    if (fast && n0 + c8 + 8 <= epi.N &&
        (epi.ones_col < 0 || n0 + c8 + 8 <= epi.ones_col))
      epi.store8_fast(gi, m0 + row, n0 + c8, v);
    else
      epi.store8(gi, m0 + row, n0 + c8, v);
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 tile, two LDS stages (2 x 64 KiB), four phases per K tile.
// Waves: group g = w >> 2 owns rows 128 g .. +128, wave w & 3 columns
// 64 (w & 3) .. +64; a wave tile is 128 x 64 (8 x 4 accumulators) split in
// quadrants of 64 x 32: q0 (A0, B0) reads A0 + B0, q1 (A0, B1) reads B1,
// q2 (A1, B1) reads A1 (into A0's registers), q3 (A1, B0) reads nothing.
// DMA per tile t, two pieces per phase: A(t+1) in q0 / q1 (its stage held
// tile t-1, fully read), B(t+2) in q2 / q3 (into tile t's stage: its B was
// last read in q1), then vmcnt(4) retires tile t+1 with B(t+2) in flight.
// Hazards by slot (group g, phase P = 4t + q: MEM slot 2P + g):
//   RAW  A(t+1) issued in slots 8t..8t+3, B(t+1) in 8t-4..8t-1, waited in
//        slots 8t+6 (g0) / 8t+7 (g1); first reads 8t+8 / 8t+9.
//   WAR  B(t+2) issued from 8t+4 after B(t)'s last read in 8t+3 (g1, q1,
//        lgkmcnt(0) before its barrier); A(t+2) from 8t+8 after A(t)'s last
//        read in 8t+5 (q2, lgkmcnt(0) before its barrier).
// The epilogue stages the f32 tile in four 64-row passes (66 KiB each).
constexpr int PQ_B = 256, PQ_SA = PQ_B * BK, PQ_SST = 2 * PQ_SA;
constexpr int PQ_LDC = PQ_B + 4;
static_assert(64 * PQ_LDC * 4 <= 2 * PQ_SST * 2, "epilogue pass fits");

template <class LP, bool PK, class LQ, bool QK>
__global__ void __launch_bounds__(512, 1)
gemm_pp256_kernel(LP lp, LQ lq, Epi epi, int P, int Q, int K, int k_split,
                  int tiles_q, int tiles, int splits, int gm) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * PQ_SST];
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = wgid % tiles;
  const int gs = wgid / tiles;
  const int gi = gs / splits;
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
  const int kbeg = (gs - gi * splits) * k_split;
  const int kend = min(K, kbeg + k_split);
  if (kbeg >= kend) return;
  lp.group(gi);
  lq.group(gi);
  const int p0 = tp * PQ_B, q0 = tq * PQ_B;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int grp = w >> 2;
  const int prow = grp * 128;        // wave's first P row
  const int qrow = (w & 3) * 64;     // wave's first Q row
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  PPOp<LP, PK, PQ_B> op;
  PPOp<LQ, QK, PQ_B> oq;
  op.init(lp, p0, w, lane, kbeg);
  oq.init(lq, q0, w, lane, kbeg);
  static_assert(PPOp<LP, PK, PQ_B>::NS == 4 && PPOp<LQ, QK, PQ_B>::NS == 4,
                "four pieces per operand and tile");
  // half h (0 / 1) of an operand's four pieces: pieces 2h, 2h + 1
  auto issue_half = [&](auto& o, const auto& l, int k0, uint16_t* s, int h) {
    o.issue_part(l, k0, s, w, 2 * h, 2);
  };

  const int nk = (kend - kbeg + BK - 1) / BK;
  uint16_t* st0 = smem;
  uint16_t* st1 = smem + PQ_SST;
  // prologue: A(0), B(0), B(1); wait for tile 0
  op.issue(lp, kbeg, st0, w);
  oq.issue(lq, kbeg, st0 + PQ_SA, w);
  if (nk > 1) {
    oq.issue(lq, kbeg + BK, st1 + PQ_SA, w);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // stagger group 1 by one slot
  asm volatile("" ::: "memory");

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  auto mfma = [&](int abase, bf16x8 (&bf)[2][2], int bbase) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[abase + i][bbase + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              af[i][ks], bf[j][ks], acc[abase + i][bbase + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto slot_end = [&]() {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int kt = 0; kt < nk; ++kt) {
    const uint16_t* sP = (kt & 1) ? st1 : st0;
    const uint16_t* sQ = sP + PQ_SA;
    uint16_t* nxt = (kt & 1) ? st0 : st1;   // tile t+1's stage
    uint16_t* cur = (kt & 1) ? st1 : st0;   // tile t+2's stage
    const bool pa = kt + 1 < nk, pb = kt + 2 < nk;
    const int ka = kbeg + (kt + 1) * BK, kb = kbeg + (kt + 2) * BK;
    // ---- q0 MEM: A0, B0; A(t+1) pieces 0, 1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b0[j][ks] = pp_frag<QK>(sQ, qrow + j * 16, ks, fr, fq);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = pp_frag<PK>(sP, prow + i * 16, ks, fr, fq);
    }
    if (pa) issue_half(op, lp, ka, nxt, 0);
    slot_end();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma(0, b0, 0);                       // q0 MFMA
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // ---- q1 MEM: B1; A(t+1) pieces 2, 3; B reads of this tile retired
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b1[j][ks] = pp_frag<QK>(sQ, qrow + 32 + j * 16, ks, fr, fq);
    if (pa) issue_half(op, lp, ka, nxt, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    slot_end();
    mfma(0, b1, 2);                       // q1 MFMA
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // ---- q2 MEM: A1; B(t+2) pieces 0, 1; A reads of this tile retired
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = pp_frag<PK>(sP, prow + 64 + i * 16, ks, fr, fq);
    if (pb) issue_half(oq, lq, kb, cur + PQ_SA, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    slot_end();
    mfma(4, b1, 2);                       // q2 MFMA
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
    // ---- q3 MEM: B(t+2) pieces 2, 3; wait for tile t+1
    if (pb) {
      issue_half(oq, lq, kb, cur + PQ_SA, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    slot_end();
    mfma(4, b0, 0);                       // q3 MFMA
    __builtin_amdgcn_sched_barrier(0);
    slot_end();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // group 1's last slot
  asm volatile("" ::: "memory");

  // epilogue: four passes of 64 rows; pass e holds group e / 2's m-tiles
  // 4 (e % 2) .. +3
  float* sC = (float*)smem;
  constexpr int CH = PQ_B / 8;
  const bool fast = epi.fast_ok();
  // (unrolled: the accumulator indices must be compile-time constants, or
  // acc goes to scratch)
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
          for (int rr = 0; rr < 4; ++rr) {
            sC[(rb + rr) * PQ_LDC + qc] = acc[(e & 1) * 4 + i][j][rr];
          }
        }
    }
    __syncthreads();
    const int m0 = p0 + e * 64;
    if (epi.atomic) {
      const int c = t & 255;
      for (int row = t >> 8; row < 64; row += 2)
        epi.store(gi, m0 + row, q0 + c, sC[row * PQ_LDC + c]);
      continue;
    }
    for (int q = t; q < 64 * CH; q += 512) {
      const int row = q / CH, c8 = (q % CH) * 8;
      if (m0 + row >= epi.M) continue;
      const float4* src = (const float4*)(sC + row * PQ_LDC + c8);
      float v[8];
      const float4 lo = src[0], hi = src[1];
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      if (fast && q0 + c8 + 8 <= epi.N &&
          (epi.ones_col < 0 || q0 + c8 + 8 <= epi.ones_col))
        epi.store8_fast(gi, m0 + row, q0 + c8, v);
      else
        epi.store8(gi, m0 + row, q0 + c8, v);
    }
  }
}

// The ping-pong loop takes a dense NT / NN GEMM (buffer-DMA operands) with
// a 128-wide column tile and at least one 256 x 128 tile per CU (one
// workgroup per CU).  hvk_gemm_variant 30 (or 0) disables it, 31 runs
// its no-DMA ablation (A/B runs).
template <class LA, bool AK, class LB, bool BKM>
bool want_pp(const LA& la, const LB& lb, int M, int N, int bn, int splits,
             int groups) {
  if constexpr (!pp_loader_ok<LA, AK, true>() ||
                !pp_loader_ok<LB, BKM, false>()) {
    return false;
  } else {
    if (hvk_gemm_variant == 30 || hvk_gemm_variant == 0) return false;
    if (bn != 128 || !la.dma_ok() || !lb.dma_ok()) return false;
    return (long long)((M + PP_BM - 1) / PP_BM) * ((N + PP_BN - 1) / PP_BN) *
               splits * groups >= 256;
  }
}

// the 256 x 256 loop where the output is wide and tall enough: at most 1/8
// of a 256 column tile wasted, and a 256 x 256 tile per CU - or fewer tiles
// than CUs when that still finishes first: in units of one 256 x 128 tile
// at the measured loop rates (1.42 vs 1.19 PF, profiles/ab_gemm_pp256_r3.log)
// ceil(t256 / 256) rounds cost 2 / 1.42 each, ceil(t128 / 256) 1 / 1.19 (AlexNet
// b1024 fc6 backward-data: 144 tiles in one round against 288 in two);
// variant 32 keeps 256 x 128 (A/B runs)
inline bool want_pp256(int M, int N, int splits, int groups) {
  if (hvk_gemm_variant == 32) return false;
  const int wn = (N + 255) / 256 * 256 - N;
  if (N < 256 || wn * 8 > N) return false;
  const long long t256 =
      (long long)((M + 255) / 256) * ((N + 255) / 256) * splits * groups;
  if (t256 >= 256) return true;
  const long long t128 =
      (long long)((M + 255) / 256) * ((N + 127) / 128) * splits * groups;
  return (t256 + 255) / 256 * 2 * 119 < (t128 + 255) / 256 * 142;
}

template <class LP, bool PK, class LQ, bool QK>
hipError_t go_pp256(const LP& lp, const LQ& lq, const Epi& epi, int P, int Q,
                    int K, int k_split, int splits, int groups,
                    hipStream_t s) {
  const int tiles_p = (P + 255) / 256, tiles_q = (Q + 255) / 256;
  const int tiles = tiles_p * tiles_q;
  const int gm = (tiles_q >= 8 && hvk_gemm_variant != 20) ? 8 : 1;
  dim3 grid((unsigned)((long long)tiles * splits * groups));
  hipLaunchKernelGGL((gemm_pp256_kernel<LP, PK, LQ, QK>), grid, dim3(512), 0,
                     s, lp, lq, epi, P, Q, K, k_split, tiles_q, tiles, splits,
                     gm);
  return launch_status(s);
}

template <class LP, bool PK, class LQ, bool QK>
hipError_t go_pp(const LP& lp, const LQ& lq, const Epi& epi, int P, int Q,
                 int K, int k_split, int splits, int groups, hipStream_t s) {
  if (want_pp256(P, Q, splits, groups))
    return go_pp256<LP, PK, LQ, QK>(lp, lq, epi, P, Q, K, k_split, splits,
                                    groups, s);
  const int tiles_p = (P + PP_BM - 1) / PP_BM;
  const int tiles_q = (Q + PP_BN - 1) / PP_BN;
  const int tiles = tiles_p * tiles_q;
  const int gm = (tiles_q >= 8 && hvk_gemm_variant != 20) ? 8 : 1;
  dim3 grid((unsigned)((long long)tiles * splits * groups));
  if constexpr (QK) {
    if (hvk_gemm_variant == 31) {
      hipLaunchKernelGGL((gemm_pp_kernel<LP, PK, LQ, QK, 1>), grid, dim3(512),
                         0, s, lp, lq, epi, P, Q, K, k_split, tiles_q, tiles,
                         splits, gm);
      return launch_status(s);
    }
  }
  hipLaunchKernelGGL((gemm_pp_kernel<LP, PK, LQ, QK>), grid, dim3(512), 0, s,
                     lp, lq, epi, P, Q, K, k_split, tiles_q, tiles, splits, gm);
  return launch_status(s);
}
