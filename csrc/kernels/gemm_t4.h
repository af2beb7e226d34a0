// gemm_t4.h - 192 x 128 tiles at TWO workgroups per CU for the
// implicit-GEMM convolutions.  Included by gemm_core.h inside its anonymous
// namespace, after gemm_pp.h.
//
// Why: the convolutions' GEMMs are short along K (AlexNet: 19-36 K tiles of
// 64) and narrow (128-384 output channels per group).  The 128 x 128 loop of
// gemm_kernel (8 waves of 64 x 32) moves 0.0156 operand bytes per FLOP and
// pays two barriers and four LDS-DMA pieces per 16 MFMAs of each wave: it is
// bound by DMA issue and synchronisation (profiles/r3_experiments.md §10).
// The one-workgroup-per-CU ping-pong loops (gemm_pp.h) move fewer bytes but
// cannot hide a tile's prologue and epilogue (§12, §13).  This loop keeps
// two independent workgroups per CU and gives each wave a 96 x 64 tile:
//
//   * 4 waves (one per SIMD) per workgroup, 2 x 2, each 96 x 64 (6 x 4
//     accumulators of MFMA 16x16x32); the other workgroup on the CU supplies
//     the second wave per SIMD, so one workgroup's barrier waits, prologue
//     and epilogue run under the other one's MFMAs;
//   * BK = 64, two LDS stages of (192 + 128) x 64 bf16 = 40 KiB: the two
//     workgroups take the whole 160 KiB.  Step t + 1 is issued at the top of
//     step t and retired at its end, ONE s_barrier per K step (48 MFMAs per
//     wave, 10 LDS-DMA pieces, 20 fragment reads);
//   * 0.013 operand bytes per FLOP (0.0156 for 128 x 128), and every K-major
//     DMA piece reads whole 128-B lines (8 rows x 64 k).
//
// Measured first with BK = 32 / 256 x 128 / three 24-KiB stages
// (profiles/r4/ab_t4_256x128_bk32_vs_128row.log): a 32-deep K-major step reads
// half of each 128-B line per row, so the L2 serves twice the requests per
// byte, and the convolutions gained at most 6 % (conv3 forward) - rejected.
// The BK template parameter keeps that configuration for A/B builds.
//
// Operand images (lane-linear LDS-DMA from pre-permuted source offsets, as
// in gemm_kernel):
//   K-major [rows][64 k], 128-B rows, 16-B chunk c of row r at c ^ (r & 7)
//     (BK 32: [rows][32 k], chunk c at c ^ t4_sw(r));
//   MN-major [64 k][IMG cols] (IMG = 128, 192), 32-B block b of k-row k at
//     b ^ t4_mnsw(k), read by ds_read_b64_tr_b16.
// The MFMA accumulation order over K is the 128-row loop's (k ascending in
// steps of 32): results are bit-identical to gemm_kernel.
//
// Orientation: the 192-row operand P and the 128-row operand Q are either
// (A, B) - C[P][Q] - or (B, A) with TRANS - C[Q][P]; the epilogue stages the
// f32 tile through the drained ring in two passes of 96 rows of P,
// transposed for TRANS, so stores (and split-K atomics) always run along
// C's contiguous dimension.

constexpr int T4_QR = 128;

// Diagnostic builds only (tools/build_abl.py; wrong results by design): bit 1
// skips the main loop's LDS-DMA, bit 2 the epilogue (the accumulators are
// kept live by a never-taken store), bit 4 the main loop's waits and
// barriers, bit 8 re-reads the first K step's sources every step (the same
// LDS-DMA traffic, all of it L1 / L2 hits), bit 16 as 8 for the im2col
// operands with the addresses computed once (no per-step addressing VALU).
#ifndef HVK_T4_ABL
#define HVK_T4_ABL 0
#endif

__device__ __forceinline__ int t4_sw(int r) {
  return (0x78 >> (2 * ((r >> 2) & 3))) & 3;
}
// MN-major images: XOR mask of k-row k's 32-B blocks.  Pitch 256 / 512 B
// (128 / 256 columns): hk(k), 8 distinct slots for the k-rows {0..3, 8..11}
// a ds_read_b64_tr_b16 lane group reads; pitch 384 B (192 columns): rows
// alternate between two bank halves, the 2-bit mask (XOR inside a group of
// four blocks, so a block never leaves its row) separates the four rows of
// each half
template <int IMG>
__device__ __forceinline__ int t4_mnsw(int k) {
  if constexpr (IMG == 192) return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  else return hk(k);
}

// One operand's DMA slots (ROWS = rows of the operand the tile computes,
// BKT = K step: 32 (three stages) or 64 (two stages))
template <class L, bool KM, int ROWS, int BKT>
struct T4Op {
  static constexpr int IMG = ROWS;
  static constexpr int NP = IMG * BKT / 512;   // 1-KiB pieces per stage
  static constexpr int NS = NP / 4;            // per wave
  static_assert(NS * 4 == NP, "pieces divide over the four waves");
  static constexpr bool FAST = L::kFast;
  static constexpr bool BUF = L::kBuf;
  __amdgpu_buffer_rsrc_t rs;
  uint32_t v[NS];
  int kr[NS];
  int kc;
  DRow fa[KM && FAST ? NS : 1];
  typename DColOf<L, !KM && FAST>::type fb[!KM && FAST ? NS : 1];
  // ABL 16 (diagnostic): the first step's sources, reused every step
  uint32_t v0[(HVK_T4_ABL & 16) && KM && FAST ? NS : 1];
  const uint16_t* p0[(HVK_T4_ABL & 16) && !KM && FAST ? NS : 1];

  __device__ __forceinline__ void init(const L& l, int r0, int kbeg, int w,
                                       int lane) {
    if constexpr (BUF) rs = dma_rsrc(l.dbase());
    if constexpr (KM) {
      // BKT 32: a piece is 16 rows x 64 B, lane L -> row L >> 2, chunk L & 3;
      // BKT 64: 8 rows x 128 B (whole cache lines), row L >> 3, chunk L & 7
      constexpr int RPP = 64 / (BKT / 8);
      constexpr int CPRW = BKT / 8;
      kc = BKT == 32 ? 8 * ((lane & 3) ^ t4_sw(lane >> 2))
                     : 8 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int row = r0 + RPP * (w * NS + i) + lane / CPRW;
        if constexpr (FAST) fa[i] = l.drow(row);
        else v[i] = l.row_voff(row);
      }
      if constexpr ((HVK_T4_ABL & 16) && FAST) {
        const DTap tp = l.dtap(kbeg + kc);
#pragma unroll
        for (int i = 0; i < NS; ++i) v0[i] = l.dvoff(fa[i], tp);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int off = (w * NS + i) * 1024 + 16 * lane;   // image byte
        kr[i] = off / (IMG * 2);
        const int pc = (off - kr[i] * IMG * 2) >> 4;        // 16-B chunk
        const int c = 16 * ((pc >> 1) ^ t4_mnsw<IMG>(kr[i])) + 8 * (pc & 1);
        if constexpr (FAST) fb[i] = l.dcol(r0 + c, kbeg + kr[i], false);
        else v[i] = l.col_voff(r0 + c, kr[i]);
        if constexpr ((HVK_T4_ABL & 16) && FAST) p0[i] = l.dsrc(fb[i]);
      }
    }
  }
  // the K step at k0 into stage s (FAST MN-major slots track k0 themselves:
  // steps must be issued in order)
  __device__ __forceinline__ void issue(const L& l, int k0, uint16_t* s,
                                        int w) {
    if constexpr ((HVK_T4_ABL & 16) && FAST) {
      // diagnostic: the same LDS-DMA traffic without per-step addressing
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        if constexpr (KM) {
          dma16(rs, s + (w * NS + i) * 512, v0[i]);
        } else {
          __builtin_amdgcn_global_load_lds(
              (const void*)p0[i],
              (__attribute__((address_space(3))) void*)(s + (w * NS + i) * 512),
              16, 0, 0);
        }
      }
      return;
    }
    if constexpr (KM && FAST) {
      const DTap tp = l.dtap(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, s + (w * NS + i) * 512, l.dvoff(fa[i], tp));
    } else if constexpr (KM) {
      const bool kin = k0 + kc < l.K;
      const uint32_t kbyte = 2u * (uint32_t)(k0 + kc);
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, s + (w * NS + i) * 512, kin ? v[i] + kbyte : kBufOOB);
    } else if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        __builtin_amdgcn_global_load_lds(
            (const void*)l.dsrc(fb[i]),
            (__attribute__((address_space(3))) void*)(s + (w * NS + i) * 512),
            16, 0, 0);
        l.dnext_by(fb[i], BKT);
      }
    } else {
      const uint32_t kadv = (uint32_t)k0 * (uint32_t)l.ld * 2u;
#pragma unroll
      for (int i = 0; i < NS; ++i)
        dma16(rs, s + (w * NS + i) * 512,
              k0 + kr[i] < l.K ? v[i] + kadv : kBufOOB);
    }
  }
};

// fragment of the 16-row MFMA tile at `row` (16-row aligned), 32-deep k
// half ks of the stage
template <bool KM, int IMG, int BKT>
__device__ __forceinline__ bf16x8 t4_frag(const uint16_t* s, int row, int ks,
                                          int fr, int fq) {
  if constexpr (KM) {
    const int r = row + fr;
    if constexpr (BKT == 32)
      return *(const bf16x8*)(s + r * 32 + ((fq ^ t4_sw(r)) << 3));
    else
      return *(const bf16x8*)(s + r * 64 + (((ks * 4 + fq) ^ (r & 7)) << 3));
  } else {
    const int b = row >> 4;
    const int trq = fr >> 2, trp = fr & 3;
    const int k = ks * 32 + fq * 8 + trq;
    const uint16_t* p0 =
        s + k * IMG + ((b ^ t4_mnsw<IMG>(k)) << 4) + trp * 4;
    const uint16_t* p1 =
        s + (k + 4) * IMG + ((b ^ t4_mnsw<IMG>(k + 4)) << 4) + trp * 4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

// BIAS (weight gradients): the bias gradient sum_k of one operand's
// columns, from extra MFMAs against an all-ones operand in the first tile
// of the other side instead of a ones column appended to the GEMM (which
// costs a whole extra tile when KK fills the tiles: AlexNet conv5 1728 =
// 9 x 192).  1: over the Q operand (ones as A; waves with prow = 0 of the
// workgroups with tp = 0); 2: over the P operand (ones as B; waves with
// qrow = 0 of the workgroups with tq = 0).  bgrad[row + gi * grow] is
// stored (bg_store, an unsplit overwrite) or atomically added.
//
// QR = 64 (outputs of 33-64 channels per group: AlexNet conv2 backward-data,
// VGG conv1_2 / conv2_1 backward-data): PR = 256 and the four waves stacked
// along P (64 x 64 each, NJ = 3 computed n-tiles for <= 48 columns) - the
// same 40-KiB stage; orientation 1 only, no bias MFMAs, staged epilogue.
template <class LP, bool PK, class LQ, bool QK, int PR, bool TRANS, int BKT,
          int BIAS = 0, int EP = 0, int QR = T4_QR, int NJ = 4>
__global__ void __launch_bounds__(256, 2)
gemm_t4_kernel(LP lp, LQ lq, Epi epi, int P, int Q, int K, int k_split,
               int tiles_q, int tiles, int splits, int gm, float* bgrad,
               int bg_store) {
  constexpr bool STK = QR == 64;             // waves stacked along P
  static_assert(!STK || (!TRANS && BIAS == 0 && EP == 0 && PR == 256),
                "stacked waves: orientation 1, staged epilogue");
  constexpr int NST = BKT == 32 ? 3 : 2;     // LDS ring stages
  using OP = T4Op<LP, PK, PR, BKT>;
  using OQ = T4Op<LQ, QK, QR, BKT>;
  constexpr int SP = OP::IMG * BKT, SQ = OQ::IMG * BKT;
  constexpr int SST = SP + SQ;
  constexpr int RING = NST * SST * 2;
  constexpr int HP = PR / 2;                 // P rows per epilogue pass
  constexpr int LDC = TRANS ? HP + 4 : QR + 4;
  constexpr int EPI = (TRANS ? QR : HP) * LDC * 4;
  constexpr int SMEM = RING > EPI ? RING : EPI;
  static_assert(2 * SMEM <= 160 * 1024, "two workgroups per CU");
  constexpr int MI = STK ? PR / 64 : PR / 32;   // m-tiles per wave
  constexpr int NSW = OP::NS + OQ::NS;       // DMA pieces per wave and step
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM / 2];

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
  const int split = gs - gi * splits;
  const int kbeg = split * k_split;
  const int kend = min(K, kbeg + k_split);
  if (kbeg >= kend) return;
  lp.group(gi);
  lq.group(gi);
  const int p0 = tp * PR, q0 = tq * QR;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int prow = STK ? w * (PR / 4) : (w >> 1) * HP;   // first P row
  const int qrow = STK ? 0 : (w & 1) * 64;               // first Q row
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NBA = BIAS == 1 ? 4 : (BIAS == 2 ? MI : 1);
  f32x4 accb[NBA];
#pragma unroll
  for (int i = 0; i < NBA; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool bwave = BIAS == 1 ? (tp == 0 && prow == 0)
                   : BIAS == 2 ? (tq == 0 && qrow == 0) : false;
  const bf16x8 ones = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                       (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f};

  OP op;
  OQ oq;
  op.init(lp, p0, kbeg, w, lane);
  oq.init(lq, q0, kbeg, w, lane);

  const int nk = (kend - kbeg + BKT - 1) / BKT;
  // prologue: NST - 1 steps in flight, wait for step 0
  op.issue(lp, kbeg, smem, w);
  oq.issue(lq, kbeg, smem + SP, w);
  if (NST == 3 && nk > 1) {
    op.issue(lp, kbeg + BKT, smem + SST, w);
    oq.issue(lq, kbeg + BKT, smem + SST + SP, w);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NSW) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // the main loop, unswitched on the wave-uniform bias flag: a branch around
  // the bias MFMAs inside the loop split it into one basic block per m-tile
  // and serialised the MFMA schedule (BIAS variants only)
  auto main_loop = [&](auto with_bias) {
    constexpr bool WB = decltype(with_bias)::value;
    int scur = 0, spre = NST - 1;  // stage of step t, of step t + NST - 1
    for (int kt = 0; kt < nk; ++kt) {
      const uint16_t* sP = smem + scur * SST;
      const uint16_t* sQ = sP + SP;
      // step t + NST - 1 into the stage step t - 1 used (every wave finished
      // reading it before the barrier that ended step t - 1)
      const bool pre = kt + NST - 1 < nk;
      if (pre && !(HVK_T4_ABL & 1)) {
        uint16_t* d = smem + spre * SST;
        const int k2 = (HVK_T4_ABL & 8) ? kbeg
                                        : kbeg + (kt + NST - 1) * BKT;
        op.issue(lp, k2, d, w);
        oq.issue(lq, k2, d + SP, w);
      }
#pragma unroll
      for (int ks = 0; ks < BKT / 32; ++ks) {
        bf16x8 bq[4];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          bq[j] = t4_frag<QK, OQ::IMG, BKT>(sQ, qrow + j * 16, ks, fr, fq);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bf16x8 a = t4_frag<PK, OP::IMG, BKT>(sP, prow + i * 16, ks,
                                                     fr, fq);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            // EP 1 / 2: the transposed product (a lane then holds 4
            // consecutive C columns of one row); same K order, same values
            if constexpr (EP != 0 && !TRANS)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  bq[j], a, acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  a, bq[j], acc[i][j], 0, 0, 0);
          }
          if constexpr (WB && BIAS == 2)
            accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ones,
                                                              accb[i], 0, 0, 0);
        }
        if constexpr (WB && BIAS == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bq[j],
                                                              accb[j], 0, 0, 0);
        }
      }
      // retire step t + 1 (three stages: step t + 2 stays in flight), then
      // one barrier: step t + 1 visible to every wave, every read of step t
      // done
      if constexpr (!(HVK_T4_ABL & 4)) {
        if (NST == 3 && pre)
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NSW) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      asm volatile("" ::: "memory");
      scur = scur == NST - 1 ? 0 : scur + 1;
      spre = spre == NST - 1 ? 0 : spre + 1;
    }
  };
  if (BIAS != 0 && bwave)
    main_loop(std::integral_constant<bool, BIAS != 0>{});
  else
    main_loop(std::false_type{});

  if constexpr ((HVK_T4_ABL & 2) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1234.5f && P < 0) epi.store(0, 0, 0, sum);
    return;
  }
  if constexpr (EP == 1) {
    // direct epilogue (no atomics, slices, fp8 copy or bias column): every
    // lane stores its accumulator quads as 4 consecutive columns of a C row
    // - no LDS staging, no barriers
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = TRANS ? q0 + qrow + j * 16 + fr : p0 + prow + i * 16 + fr;
        const int n = TRANS ? p0 + prow + i * 16 + fq * 4
                            : q0 + qrow + j * 16 + fq * 4;
        if (m < epi.M && n < epi.N) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2],
                        acc[i][j][3]};
          epi.store4_fast(gi, m, n, v);
        }
      }
    return;
  }
  if constexpr (EP == 2) {
    // register epilogue: each lane finishes its accumulator quads (4
    // consecutive C columns of one row: alpha, bias, activation, derivative
    // of the layer below, bf16) and writes 8 B into a bf16 image of the
    // whole C tile in the drained ring (one pass, 48 KiB); then whole 16-B
    // row chunks go out as in the staged epilogue (and the fp8 copy).  A
    // quarter of the LDS traffic and of the epilogue VALU of the f32 staging
    constexpr int OR_ = TRANS ? T4_QR : PR;      // C rows of the tile
    constexpr int OC_ = TRANS ? PR : T4_QR;      // C columns
    constexpr int LDO = OC_ + 8;                 // bf16 elements per row
    static_assert(OR_ * LDO * 2 <= RING, "bf16 C tile fits the ring");
    uint16_t* sO = smem;
    const int m0 = TRANS ? q0 : p0, n0 = TRANS ? p0 : q0;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = TRANS ? qrow + j * 16 + fr : prow + i * 16 + fr;
        const int nl = TRANS ? prow + i * 16 + fq * 4 : qrow + j * 16 + fq * 4;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        uint2 o = make_uint2(0u, 0u);
        if (m0 + ml < epi.M && n0 + nl < epi.N)
          o = epi.pre4(gi, m0 + ml, n0 + nl, v);
        *(uint2*)(sO + ml * LDO + nl) = o;
      }
    __syncthreads();
    const float qs = epi.q8.q ? fp8_scale(epi.q8.st, epi.q8.hist, epi.q8.fmax)
                              : 1.f;
    float amax = 0.f;
    constexpr int CH = OC_ / 8;
    for (int q = t; q < OR_ * CH; q += 256) {
      const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
      if (m0 + row >= epi.M || n0 + c8 >= epi.N) continue;
      const uint4 ob = *(const uint4*)(sO + row * LDO + c8);
      const long long idx = (long long)(m0 + row + gi * epi.grow) * epi.ldc +
                            n0 + c8 + gi * epi.gcol;
      *(uint4*)((uint16_t*)epi.c + idx) = ob;
      if (epi.q8.q) q8_store8(epi.q8, idx, ob, qs, amax);
    }
    if (epi.q8.q) {  // block-uniform
      __syncthreads();   // sO reads done: its first words hold the reduction
      q8_block_amax(epi.q8, amax, (float*)smem);
    }
    return;
  }
  if constexpr (BIAS != 0) {
    // every row (BIAS 1) / column (BIAS 2) of the ones-MFMA tile holds the
    // same sums: lanes of row 0 / column 0 write them
    if (bwave) {
      const int eg0 = epi.slice ? 0 : gi;
#pragma unroll
      for (int i = 0; i < NBA; ++i) {
        if constexpr (BIAS == 1) {
          const int r = q0 + qrow + i * 16 + fr;      // Q index = C row
          if (fq == 0 && r < Q) {
            const float v = accb[i][0] * epi.alpha;
            float* d = bgrad + r + eg0 * epi.grow;
            if (bg_store) *d = v;
            else atomicAdd(d, v);
          }
        } else {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int r = p0 + prow + i * 16 + fq * 4 + rr;  // P = C row
            if (fr == 0 && r < P) {
              const float v = accb[i][rr] * epi.alpha;
              float* d = bgrad + r + eg0 * epi.grow;
              if (bg_store) *d = v;
              else atomicAdd(d, v);
            }
          }
        }
      }
    }
  }

  // epilogue: the ring is drained (every DMA waited for, every fragment read
  // consumed before the last barrier).  Two passes over the P rows; pass e
  // holds the accumulators of the waves with (w >> 1) == e.
  float* sC = (float*)smem;
  const bool fast = epi.fast_ok();
  const float qs = epi.q8.q ? fp8_scale(epi.q8.st, epi.q8.hist, epi.q8.fmax)
                            : 1.f;
  float amax = 0.f;
  const int eg = epi.slice ? split : gi;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    if (e) __syncthreads();
    if ((w >> 1) == e) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pl = prow - e * HP + i * 16 + fq * 4;  // pass-local P row
          const int qc = qrow + j * 16 + fr;               // Q row
          if constexpr (TRANS) {
            *(float4*)(sC + qc * LDC + pl) =
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2],
                            acc[i][j][3]);
          } else {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
              sC[(pl + rr) * LDC + qc] = acc[i][j][rr];
          }
        }
    }
    __syncthreads();
    // C rows / columns of this pass
    constexpr int ROWS = TRANS ? QR : HP;
    constexpr int COLS = TRANS ? HP : QR;
    const int m0 = TRANS ? q0 : p0 + e * HP;
    const int n0 = TRANS ? p0 + e * HP : q0;
    if (epi.atomic) {
      for (int q = t; q < ROWS * COLS; q += 256) {
        const int row = q / COLS, c = q - (q / COLS) * COLS;
        epi.store(eg, m0 + row, n0 + c, sC[row * LDC + c]);
      }
      continue;
    }
    constexpr int CH = COLS / 8;
    for (int q = t; q < ROWS * CH; q += 256) {
      const int row = q / CH, c8 = (q - (q / CH) * CH) * 8;
      if (m0 + row >= epi.M) continue;
      const float4* src = (const float4*)(sC + row * LDC + c8);
      float v[8];
      const float4 lo = src[0], hi = src[1];
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      if (fast && n0 + c8 + 8 <= epi.N &&
          (epi.ones_col < 0 || n0 + c8 + 8 <= epi.ones_col))
        epi.store8_fast(eg, m0 + row, n0 + c8, v, qs, &amax);
      else
        epi.store8(eg, m0 + row, n0 + c8, v);
    }
  }
  if (epi.q8.q) {  // block-uniform
    __syncthreads();   // sC reads done: its first words hold the reduction
    q8_block_amax(epi.q8, amax, sC);
  }
}

// ------------------------------------------------------------ dispatch
// The operand pairs that take the T4 loop (LDS-DMA loaders with buffer
// descriptors or the fast wgrad gather): conv forward / backward-data (A =
// implicit im2col, K-major; B = weights, K-major) and the conv weight
// gradient (A = dY MN-major, B = im2col MN-major).
template <class LA, bool AK, class LB, bool BKM>
constexpr bool t4_pair_ok() {
  if constexpr (AK && BKM)
    return std::is_same<LB, DenseK>::value &&
           (std::is_same<LA, ConvFwdA>::value ||
            std::is_same<LA, ConvDgradA>::value);
  else if constexpr (!AK && !BKM)
    return std::is_same<LA, DenseMN>::value &&
           std::is_same<LB, ConvWgradB>::value;
  else
    return false;
}

// orientation options (M = A rows, N = B rows), both 192 x 128 tiles at
// BK 64: 1 P = A, Q = B; 2 P = B, Q = A, TRANS.  Cost = padded MFMA work;
// the T4 loop is taken when its padded work is at most 1.04x (weight
// gradients: 0.90x, see t4_pick) that of the 128-row loop (which pads to
// 128 x bn tiles): measured at AlexNet b1024
// (profiles/r4/ab_t4_192x128_bk64_vs_128row.log) the forward and
// backward-data convolutions gain 3-27 % at <= 1.0x.  hvk_gemm_variant 50
// turns the loop off, 51 / 52 force option 1 / 2 (A/B runs, tests).
inline long long t4_cost(int M, int N, int opt) {
  auto up = [](long long x, long long b) { return (x + b - 1) / b * b; };
  return opt == 1 ? up(M, 192) * up(N, 128) : up(N, 192) * up(M, 128);
}

// Nt: the N the T4 tiles cover (a weight gradient's bias comes from ones-
// MFMAs instead of the ones column the 128-row loop pads N with).  pct: the
// padded-work ratio (percent) up to which T4 is taken.  Weight gradients
// need <= 0.90: at equal padding the 8-wave 128-row loop is faster on them
// (AlexNet b1024: conv3 wgrad 0.947x -> T4 825 vs 882 TF, conv5 0.964x ->
// 773 vs 839; conv4 at 0.75x gains 696 -> 855; profiles/r4/t4_ablation/).
inline int t4_pick(int M, int N, int bn, int Nt, int pct = 104) {
  if (hvk_gemm_variant == 50 || hvk_gemm_variant == 0) return 0;
  if (hvk_gemm_variant == 51) return 1;
  if (hvk_gemm_variant == 52) return 2;
  const long long c1 = t4_cost(M, Nt, 1), c2 = t4_cost(M, Nt, 2);
  const long long base = (long long)((M + 127) / 128 * 128) *
                         ((N + bn - 1) / bn * bn);
  const int best = c1 <= c2 ? 1 : 2;
  const long long cb = c1 <= c2 ? c1 : c2;
  return cb * 100 <= base * pct ? best : 0;
}

// the direct (register -> global) epilogue: one K split, plain vector
// stores (no atomics, workspace slices, fp8 copy or bias column), 4-column
// groups.  Opt-in (hvk_gemm_variant 53): measured SLOWER than the staged
// epilogue on every AlexNet / VGG conv it applies to (conv5 dgrad 967 ->
// 713 TF, conv2 fwd 834 -> 688; profiles/r4/t4_ablation/README.md): a lane's
// 8-B quads leave 32-B pieces of each output row per store instruction,
// where the staged epilogue writes whole 256-B row runs.
inline bool t4_direct_ok(const Epi& e, int splits) {
  return hvk_gemm_variant == 53 && splits == 1 && e.fast_ok() && !e.slice &&
         !e.q8.q && e.ones_col < 0 && (e.N & 3) == 0;
}

// the register epilogue with a bf16 C image (EP 2): one K split, bf16
// output written once (no beta, atomics, slices or bias column), 8-column
// groups.  Opt-in (hvk_gemm_variant 54): measured slower than the f32
// staging at AlexNet b1024 (conv4 dgrad 1025 -> 862 TF, conv5 dgrad 960 ->
// 758, conv5 fwd 901 -> 847; profiles/r4/t4_ablation/README.md) - the lane
// quads read the derivative of the layer below in 32-B pieces per row and
// write the bf16 image with 4-way bank conflicts
inline bool t4_regepi_ok(const Epi& e, int splits) {
  return hvk_gemm_variant == 54 && splits == 1 && e.fast_ok() && !e.slice &&
         !e.out_f32 && e.beta == 0.f && e.ones_col < 0 && (e.N & 7) == 0;
}

template <class LP, bool PK, class LQ, bool QK, bool TRANS, int BIAS = 0,
          int EP = 0, int QR = T4_QR, int NJ = 4>
hipError_t go_t4(const LP& lp, const LQ& lq, const Epi& epi, int P, int Q,
                 int K, int k_split, int splits, int groups, hipStream_t s,
                 float* bgrad = nullptr, int bg_store = 0) {
  constexpr int PR = QR == 64 ? 256 : 192;
  const int tiles_p = (P + PR - 1) / PR, tiles_q = (Q + QR - 1) / QR;
  const int tiles = tiles_p * tiles_q;
  const int gm = (tiles_q >= 8 && hvk_gemm_variant != 20) ? 8 : 1;
  dim3 grid((unsigned)((long long)tiles * splits * groups));
  hipLaunchKernelGGL((gemm_t4_kernel<LP, PK, LQ, QK, PR, TRANS, 64, BIAS, EP,
                                     QR, NJ>),
                     grid, dim3(256), 0, s, lp, lq, epi, P, Q, K, k_split,
                     tiles_q, tiles, splits, gm, bgrad, bg_store);
  return launch_status(s);
}

// Launch on the T4 loop if the shape takes it; *taken = false leaves the
// call to the other loops.  A split-K launch is re-split so that the T4
// tiles launch as many workgroups as the 128 x bn tiles would have.
template <class LA, bool AK, class LB, bool BKM>
hipError_t t4_launch(const LA& la, const LB& lb, const Epi& epi, int M, int N,
                     int K, int k_split, int tiles, int splits, int groups,
                     int bn, hipStream_t s, bool* taken) {
  *taken = false;
  if constexpr (!t4_pair_ok<LA, AK, LB, BKM>()) {
    return hipSuccess;
  } else {
    if (!la.dma_ok() || !lb.dma_ok()) return hipSuccess;
    if constexpr (std::is_same<LB, ConvWgradB>::value) {
      // the gather's running pixel wraps into the next image at most once
      // per 64-pixel step
      if (lb.g.OH * lb.g.OW < 64) return hipSuccess;
    }
    // weight gradient with a fused bias gradient: the bias comes from ones-
    // MFMAs (BIAS), not from the ones column at index N - 1
    const bool wbias = std::is_same<LB, ConvWgradB>::value &&
                       epi.ones_col >= 0 && epi.ones_col == N - 1;
    const int Nt = wbias ? N - 1 : N;
    if constexpr (!std::is_same<LB, ConvWgradB>::value) {
      // 33-64 output channels per group: 256 x 64 tiles with the waves
      // stacked along the pixels (the 128-row loop's VAR 3 / 4 tile shape on
      // the T4 schedule).  Opt-in (hvk_gemm_variant 58): slower than VAR 3 /
      // 4's eight waves per workgroup at AlexNet b1024 (conv2 backward-data
      // 737 -> 705 TF; profiles/r4/t4_ablation/ab_t4_64.log)
      if (N > 32 && N <= 64 && splits == 1 && !epi.slice &&
          hvk_gemm_variant == 58) {
        *taken = true;
        if (N <= 48)
          return go_t4<LA, AK, LB, BKM, false, 0, 0, 64, 3>(
              la, lb, epi, M, N, K, k_split, 1, groups, s);
        return go_t4<LA, AK, LB, BKM, false, 0, 0, 64, 4>(
            la, lb, epi, M, N, K, k_split, 1, groups, s);
      }
    }
    const int opt = t4_pick(M, N, bn, Nt,
                            std::is_same<LB, ConvWgradB>::value ? 90 : 104);
    if (!opt) return hipSuccess;
    const long long t4t = opt == 1
        ? (long long)((M + 191) / 192) * ((Nt + T4_QR - 1) / T4_QR)
        : (long long)((Nt + 191) / 192) * ((M + T4_QR - 1) / T4_QR);
    int sp = splits, ks = k_split;
    // (split-K through workspace slices keeps the caller's split: the
    // finishing pass sums exactly `splits` slices)
    if (splits > 1 && !epi.slice) {
      const long long want = ((long long)tiles * splits + t4t - 1) / t4t;
      ks = (int)((K + want - 1) / want);
      ks = (ks + 63) / 64 * 64;
      sp = (K + ks - 1) / ks;
    }
    *taken = true;
    if constexpr (std::is_same<LB, ConvWgradB>::value) {
      if (wbias) {
        LB lb2 = lb;
        lb2.ones = 0;
        Epi e2 = epi;
        e2.ones_col = -1;
        e2.N = Nt;
        // an unsplit overwrite stores the bias, else adds it (split-K /
        // accumulation; the caller zeroed it for a split overwrite)
        const int bst = (!epi.atomic && epi.bias_store) ? 1 : 0;
        if (opt == 1)
          return go_t4<LA, AK, LB, BKM, false, 2>(la, lb2, e2, M, Nt, K, ks,
                                                  sp, groups, s,
                                                  epi.bias_grad, bst);
        return go_t4<LB, BKM, LA, AK, true, 1>(lb2, la, e2, Nt, M, K, ks, sp,
                                               groups, s, epi.bias_grad, bst);
      }
    }
    if constexpr (!std::is_same<LB, ConvWgradB>::value) {
      // convolution forward / backward-data outputs: the direct epilogue
      // when selected (t4_direct_ok)
      if (t4_direct_ok(epi, sp)) {
        if (opt == 1)
          return go_t4<LA, AK, LB, BKM, false, 0, 1>(la, lb, epi, M, N, K,
                                                     ks, sp, groups, s);
        return go_t4<LB, BKM, LA, AK, true, 0, 1>(lb, la, epi, N, M, K, ks,
                                                  sp, groups, s);
      }
      if (t4_regepi_ok(epi, sp)) {
        if (opt == 1)
          return go_t4<LA, AK, LB, BKM, false, 0, 2>(la, lb, epi, M, N, K,
                                                     ks, sp, groups, s);
        return go_t4<LB, BKM, LA, AK, true, 0, 2>(lb, la, epi, N, M, K, ks,
                                                  sp, groups, s);
      }
    }
    if (opt == 1)
      return go_t4<LA, AK, LB, BKM, false>(la, lb, epi, M, N, K, ks, sp,
                                           groups, s);
    return go_t4<LB, BKM, LA, AK, true>(lb, la, epi, N, M, K, ks, sp, groups,
                                        s);
  }
}
