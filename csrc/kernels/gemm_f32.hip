// gemm_f32.hip - exact-precision GEMMs on the gfx950 matrix cores: SGEMM on
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate, bit-for-bit an fmaf
// chain) and DGEMM on v_mfma_f64_16x16x4_f64, with the reference's three
// precision levels (veles/ocl_blas.py, ocl/matrix_multiplication*.cl,
// devices/device_infos.json; docs/source/manualrst_veles_common_parameters
// .rst:36-37):
//   0  plain accumulation;
//   1  Kahan: each 32-deep (f32) / 16-deep (f64) K tile is summed by the
//      MFMAs into a fresh accumulator, and the tile sums are added to the
//      running sum with a compensation term;
//   2  Neumaier / TwoSum: the tile sums are added with an exact TwoSum whose
//      rounding errors are accumulated separately (double-word sum).
// These are the DeviceBenchmark kernels of BASELINE.md (SGEMM / DGEMM
// 3001^3) and the fp32 / fp64 path of ops.gemm.
//
// Tile 128 x 128, 4 waves of 64 x 64, K tile = 128 bytes of a row (32 f32 /
// 16 f64).  Operands are register-staged (global -> VGPR -> LDS) so that a
// transposed operand is turned K-major on the way in; LDS rows are 128 B
// with the 16-B chunk XOR swizzle c ^ (row & 7).  A lane reads 16 B of its
// row per fragment (4 f32 / 2 f64 consecutive k) and feeds element j to
// MFMA j: lane quad q covers k = 4q + j (f32) - the same permutation for A
// and B, so the sum over k is unchanged.
#include "conv_geom.h"

using namespace hvk;

typedef __attribute__((ext_vector_type(4))) double f64x4;

namespace {

constexpr int BM = 128, NTHR = 256;

template <typename T> struct Mfma;
template <> struct Mfma<float> {
  typedef f32x4 acc_t;
  static constexpr int EPC = 4;    // elements per 16-B chunk
  static constexpr int BK = 32;    // elements per 128-B row
  __device__ static acc_t run(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // C/D map: col = lane & 15, row = 4 * (lane >> 4) + r
  __device__ static int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};
template <> struct Mfma<double> {
  typedef f64x4 acc_t;
  static constexpr int EPC = 2;
  static constexpr int BK = 16;
  __device__ static acc_t run(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 r
  __device__ static int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

template <typename T>
struct Operand {
  const T* p;
  int rows, K, ld, trans;  // trans: stored [K][rows]
  __device__ __forceinline__ T at(int r, int k) const {
    if (r >= rows || k >= K) return T(0);
    return trans ? p[(long long)k * ld + r] : p[(long long)r * ld + k];
  }
};

// one 16-B chunk per (row, chunk) for K-major, per (k, row-chunk) for
// transposed operands; 4 chunks per thread per operand per K tile
template <typename T>
struct Stage {
  static constexpr int EPC = Mfma<T>::EPC, BK = Mfma<T>::BK;
  T v[4][EPC];
  __device__ void load(const Operand<T>& o, int r0, int k0, int t, int vec) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!o.trans) {
        const int r = r0 + (t >> 3) + 32 * i, k = k0 + (t & 7) * EPC;
        if (vec && r < o.rows && k + EPC <= o.K) {
          const T* src = o.p + (long long)r * o.ld + k;
          if constexpr (EPC == 4) {
            float4 f = *(const float4*)src;
            v[i][0] = f.x; v[i][1] = f.y; v[i][2] = f.z; v[i][3] = f.w;
          } else {
            double2 d = *(const double2*)src;
            v[i][0] = d.x; v[i][1] = d.y;
          }
        } else {
#pragma unroll
          for (int j = 0; j < EPC; ++j) v[i][j] = o.at(r, k + j);
        }
      } else {
        constexpr int CPR = BM / EPC;          // chunks per k row
        constexpr int RPS = NTHR / CPR;        // k rows per sweep
        const int k = k0 + t / CPR + RPS * i, r = r0 + (t % CPR) * EPC;
        if (vec && k < o.K && r + EPC <= o.rows) {
          const T* src = o.p + (long long)k * o.ld + r;
          if constexpr (EPC == 4) {
            float4 f = *(const float4*)src;
            v[i][0] = f.x; v[i][1] = f.y; v[i][2] = f.z; v[i][3] = f.w;
          } else {
            double2 d = *(const double2*)src;
            v[i][0] = d.x; v[i][1] = d.y;
          }
        } else {
#pragma unroll
          for (int j = 0; j < EPC; ++j) v[i][j] = o.at(r + j, k);
        }
      }
    }
  }
  // LDS image: [128 rows][BK] with chunk c of row r at (c ^ (r & 7))
  __device__ void store(T* s, int trans, int t) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (!trans) {
        const int r = (t >> 3) + 32 * i, c = t & 7;
        T* d = s + r * BK + ((c ^ (r & 7)) * EPC);
#pragma unroll
        for (int j = 0; j < EPC; ++j) d[j] = v[i][j];
      } else {
        constexpr int CPR = BM / EPC, RPS = NTHR / CPR;
        const int k = t / CPR + RPS * i, r0 = (t % CPR) * EPC;
        const int c = k / EPC, e = k % EPC;
#pragma unroll
        for (int j = 0; j < EPC; ++j) {
          const int r = r0 + j;
          s[r * BK + ((c ^ (r & 7)) * EPC) + e] = v[i][j];
        }
      }
    }
  }
};

template <typename T, int PL>
__global__ void __launch_bounds__(NTHR, 1)
gemm_fx_kernel(Operand<T> A, Operand<T> B, T* C, int ldc, int M, int N, int K,
               T alpha, T beta, int tiles_n, int va, int vb) {
  typedef typename Mfma<T>::acc_t acc_t;
  constexpr int EPC = Mfma<T>::EPC, BK = Mfma<T>::BK;
  constexpr int TILE = BM * BK;
  __shared__ __attribute__((aligned(16))) T smem[4 * TILE];

  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BM;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fq = lane >> 4;

  acc_t acc[4][4], sum[4][4], comp[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[i][j] = acc_t{0, 0, 0, 0};
      if constexpr (PL > 0) {
        sum[i][j] = acc_t{0, 0, 0, 0};
        comp[i][j] = acc_t{0, 0, 0, 0};
      }
    }

  auto frag = [&](const T* s, int rowbase, int g, T* out) {
    const int row = rowbase + fr;
    const int c = 4 * g + fq;
    const T* p = s + row * BK + ((c ^ (row & 7)) * EPC);
#pragma unroll
    for (int j = 0; j < EPC; ++j) out[j] = p[j];
  };
  auto compute = [&](const T* sA, const T* sB) {
#pragma unroll
    for (int g = 0; g < BK / (4 * EPC); ++g) {
      T af[4][EPC], bf[4][EPC];
#pragma unroll
      for (int i = 0; i < 4; ++i) frag(sA, wm * 64 + i * 16, g, af[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i) frag(sB, wn * 64 + i * 16, g, bf[i]);
#pragma unroll
      for (int j = 0; j < EPC; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[i][jj] = Mfma<T>::run(af[i][j], bf[jj][j], acc[i][jj]);
    }
  };
  // compensated add of this K tile's sums (levels 1 / 2)
  auto fold = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const T x = acc[i][j][r];
          const T s = sum[i][j][r];
          if constexpr (PL == 1) {       // Kahan
            const T y = x - comp[i][j][r];
            const T u = s + y;
            comp[i][j][r] = (u - s) - y;
            sum[i][j][r] = u;
          } else {                       // TwoSum (Neumaier)
            const T u = s + x;
            const T bp = u - s;
            comp[i][j][r] += (s - (u - bp)) + (x - bp);
            sum[i][j][r] = u;
          }
          acc[i][j][r] = 0;
        }
  };

  Stage<T> ra, rb;
  const int nk = (K + BK - 1) / BK;
  ra.load(A, m0, 0, t, va);
  rb.load(B, n0, 0, t, vb);
  ra.store(smem, A.trans, t);
  rb.store(smem + TILE, B.trans, t);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      ra.load(A, m0, (kt + 1) * BK, t, va);
      rb.load(B, n0, (kt + 1) * BK, t, vb);
    }
    compute(smem + cur * 2 * TILE, smem + cur * 2 * TILE + TILE);
    if constexpr (PL > 0) fold();
    if (more) {
      ra.store(smem + (cur ^ 1) * 2 * TILE, A.trans, t);
      rb.store(smem + (cur ^ 1) * 2 * TILE + TILE, B.trans, t);
    }
    __syncthreads();
    cur ^= 1;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + fr;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + Mfma<T>::row(lane, r);
        if (m >= M) continue;
        T v;
        if constexpr (PL == 0) v = acc[i][j][r];
        else if constexpr (PL == 1) v = sum[i][j][r];
        else v = sum[i][j][r] + comp[i][j][r];
        T* d = C + (long long)m * ldc + n;
        *d = beta != T(0) ? alpha * v + beta * *d : alpha * v;
      }
    }
}

template <typename T>
int launch_fx(int ta, int tb, int M, int N, int K, const T* A, int lda,
              const T* B, int ldb, T* C, int ldc, T alpha, T beta, int pl,
              hipStream_t s) {
  constexpr int EPC = Mfma<T>::EPC;
  Operand<T> oa{A, M, K, lda, ta};
  Operand<T> ob{B, N, K, ldb, tb ? 0 : 1};  // B[K][N] is "transposed" rows=N
  const int va = al16(A) && lda % EPC == 0;
  const int vb = al16(B) && ldb % EPC == 0;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BM - 1) / BM;
  dim3 grid((unsigned)(tiles_m * tiles_n));
  if (pl <= 0)
    hipLaunchKernelGGL((gemm_fx_kernel<T, 0>), grid, dim3(NTHR), 0, s, oa, ob,
                       C, ldc, M, N, K, alpha, beta, tiles_n, va, vb);
  else if (pl == 1)
    hipLaunchKernelGGL((gemm_fx_kernel<T, 1>), grid, dim3(NTHR), 0, s, oa, ob,
                       C, ldc, M, N, K, alpha, beta, tiles_n, va, vb);
  else
    hipLaunchKernelGGL((gemm_fx_kernel<T, 2>), grid, dim3(NTHR), 0, s, oa, ob,
                       C, ldc, M, N, K, alpha, beta, tiles_n, va, vb);
  return (int)launch_status(s);
}

}  // namespace

// C[M][N] = alpha * op(A) . op(B) + beta * C in f32 (exact f32 MFMA).
// transA = 0: A is [M][K]; 1: [K][M].  transB = 0: B is [K][N]; 1: [N][K].
HVK_API int hvk_gemm_f32(int transA, int transB, int M, int N, int K,
                         const float* A, int lda, const float* B, int ldb,
                         float* C, int ldc, float alpha, float beta,
                         int precision_level, hipStream_t s) {
  return launch_fx<float>(transA, transB, M, N, K, A, lda, B, ldb, C, ldc,
                          alpha, beta, precision_level, s);
}

HVK_API int hvk_gemm_f64(int transA, int transB, int M, int N, int K,
                         const double* A, int lda, const double* B, int ldb,
                         double* C, int ldc, double alpha, double beta,
                         int precision_level, hipStream_t s) {
  return launch_fx<double>(transA, transB, M, N, K, A, lda, B, ldb, C, ldc,
                           alpha, beta, precision_level, s);
}
