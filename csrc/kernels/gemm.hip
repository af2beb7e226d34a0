// gemm.hip - dense GEMM entry points (the four transpose layouts, split-K)
// and the explicit im2col; the main loop is in gemm_core.h.
#include "gemm_core.h"

int hvk_gemm_variant = -1;

namespace {

// Explicit im2col for convolutions whose channel count is not a multiple of
// 8 (AlexNet conv1, C = 3): col[m][k] with k = (kh*KW + kw)*C + c padded to
// Kp (multiple of 8) with zeros, so the GEMM reads 16-B vectors.  The same
// matrix feeds the forward GEMM and the weight-gradient GEMM.
__global__ void im2col_kernel(const uint16_t* x, uint16_t* col, ConvGeom g,
                              int M, int K, int Kp) {
  const int KC = Kp >> 3;  // 8-element chunks per row
  const long long total = (long long)M * KC;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       e < total; e += (long long)gridDim.x * blockDim.x) {
    uint32_t m = (uint32_t)(e / KC);
    int kc = (int)(e - (long long)m * KC);
    uint32_t n, rem, oh, ow;
    fdivmod(m, g.fOHOW, n, rem);
    fdivmod(rem, g.fOW, oh, ow);
    int ih0 = oh * g.sy - g.pt, iw0 = ow * g.sx - g.pl;
    const uint16_t* xb = x + (long long)n * g.H * g.W * g.C;
    uint16_t o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int k = kc * 8 + j;
      o[j] = 0;
      if (k < K) {
        uint32_t t, ch, kh, kw;
        fdivmod(k, g.fCg, t, ch);
        fdivmod(t, g.fKW, kh, kw);
        int ih = ih0 + (int)kh, iw = iw0 + (int)kw;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          o[j] = xb[(ih * g.W + iw) * g.C + ch];
      }
    }
    *(uint4*)(col + (long long)m * Kp + kc * 8) = *(uint4*)o;
  }
}

// Split-K finishing pass: C = epilogue(sum of the K splits' slices of ws),
// summed in split order (deterministic; N % 8 == 0 and Epi::fast_ok(): one
// 8-column chunk per thread)
__global__ void splitk_finish_kernel(const float* __restrict__ ws, int M,
                                     int N, int splits, Epi e) {
  const int CH = N >> 3;
  const long long total = (long long)M * CH;
  const long long slice = (long long)M * N;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       q < total; q += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(q / CH), c8 = (int)(q - (long long)m * CH) * 8;
    const float4* src = (const float4*)(ws + (long long)m * N + c8);
    float4 lo = src[0], hi = src[1];
    for (int sp = 1; sp < splits; ++sp) {
      const float4* p = (const float4*)((const float*)src + sp * slice);
      const float4 a = p[0], b = p[1];
      lo.x += a.x; lo.y += a.y; lo.z += a.z; lo.w += a.w;
      hi.x += b.x; hi.y += b.y; hi.z += b.z; hi.w += b.w;
    }
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    e.store8_fast(0, m, c8, v);
  }
}

// the four operand orientations of hvk_gemm on one epilogue
hipError_t gemm_dispatch(int transA, int transB, int M, int N, int K,
                         const uint16_t* a, int lda, const uint16_t* b,
                         int ldb, const Epi& e, int splits, int oc,
                         hipStream_t s) {
  const int Nk = oc >= 0 ? N + 1 : N;
  const int va = al16(a) && (lda % 8 == 0), vb = al16(b) && (ldb % 8 == 0);
  if (!transA && transB) {
    DenseK la{a, 0, M, K, lda, va};
    DenseK lb{b, 0, N, K, ldb, vb};
    return launch<DenseK, true, DenseK, true>(la, lb, e, M, N, K, splits, 1, s);
  }
  if (!transA && !transB) {
    DenseK la{a, 0, M, K, lda, va};
    DenseMN lb{b, 0, N, K, ldb, vb, oc};
    return launch<DenseK, true, DenseMN, false>(la, lb, e, M, Nk, K, splits, 1,
                                                s);
  }
  if (transA && !transB) {
    DenseMN la{a, 0, M, K, lda, va, -1};
    DenseMN lb{b, 0, N, K, ldb, vb, oc};
    return launch<DenseMN, false, DenseMN, false>(la, lb, e, M, Nk, K, splits,
                                                  1, s);
  }
  DenseMN la{a, 0, M, K, lda, va, -1};
  DenseK lb{b, 0, N, K, ldb, vb};
  return launch<DenseMN, false, DenseK, true>(la, lb, e, M, N, K, splits, 1, s);
}

}  // namespace

HVK_API void hvk_set_gemm_variant(int v) { hvk_gemm_variant = v; }

// Returns and clears this thread's pending HIP error.  The entry points
// report launch_status(s) after their launches, so an error left pending by
// an earlier runtime call (a graph capture that was invalidated and then
// abandoned: hipErrorStreamCaptureInvalidated) would otherwise be charged to
// the next kernel launched; graphs.py drains it after a failed capture.
HVK_API int hvk_take_last_error() { return (int)hipGetLastError(); }

// A non-blocking stream of the library's own (graphs.py captures on it, via
// torch.cuda.ExternalStream): a capture stream broken by a failed capture
// is dropped for good instead of going back to torch's stream pool.
HVK_API void* hvk_stream_create() {
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return nullptr;
  return (void*)s;
}

// Ends a stream capture that failed (its graph is discarded): a capture
// whose capture_end raised can leave the stream in the capture state, and
// torch hands pooled streams out again - a later "new" stream that is still
// capturing fails every launch with hipErrorStreamCaptureInvalidated.
// Returns 1 if a capture was ended, 0 if none was in progress.
HVK_API int hvk_end_stream_capture(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) (void)hipGetLastError();
  if (st == hipStreamCaptureStatusNone) return 0;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(s, &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return 1;
}

// col[M][Kp] = im2col(X) for a single-group conv (Kp = round_up(KH*KW*C, 8))
HVK_API int hvk_im2col(const void* X, void* col, int N, int H, int W, int C,
                       int KH, int KW, int sy, int sx, int pt, int pl, int OH,
                       int OW, int Kp, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, C, KH, KW, sy, sx, pt, pl, OH, OW, 1);
  int M = N * OH * OW, K = KH * KW * C;
  long long total = (long long)M * (Kp / 8);
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(im2col_kernel, dim3((int)blocks), dim3(256), 0, s,
                     (const uint16_t*)X, (uint16_t*)col, g, M, K, Kp);
  return (int)launch_status(s);
}

// C[M][N] = alpha*op(A)*op(B) + beta*C (+bias, act, aux-derivative mask)
// transA=0: A is [M][K] (lda); transA=1: A is [K][M].
// transB=0: B is [K][N] (ldb); transB=1: B is [N][K].
// bias_grad (optional, requires transB == 0 and atomic): a ones column is
// appended to B so bias_grad[m] += sum_k A[m][k] comes out of the same GEMM.
HVK_API int hvk_gemm(int transA, int transB, int M, int N, int K,
                     const void* A, int lda, const void* B, int ldb, void* C,
                     int ldc, int out_f32, int atomic, float alpha, float beta,
                     const float* bias, int bias_mode, int act, const void* aux,
                     int ld_aux, int aux_act, int splits, float* bias_grad,
                     hipStream_t s) {
  if (bias_grad && (transB || !atomic)) return -2;
  const int Nk = bias_grad ? N + 1 : N;
  Epi e = make_epi(C, ldc, M, Nk, out_f32, atomic, alpha, beta, bias,
                   bias_mode, act, aux, ld_aux, aux_act);
  if (bias_grad) {
    e.ones_col = N;
    e.bias_grad = bias_grad;
  }
  return (int)gemm_dispatch(transA, transB, M, N, K, (const uint16_t*)A, lda,
                            (const uint16_t*)B, ldb, e, splits,
                            bias_grad ? N : -1, s);
}

// Split-K GEMM for shapes with too few output tiles to fill 256 CUs (the FC
// layers at batch 512: fc6 forward is 4 x 32 tiles of 128 x 128): the K range
// is split `splits` ways, each split STORES its partial product to its own
// slice of the workspace ws[splits][M][N] (no f32 atomics, no zeroing), then
// one pass sums the slices in split order and applies alpha, the per-column
// bias, the activation and the aux derivative and casts to C.  ws holds
// splits * M * N floats.  Same arguments as hvk_gemm minus beta /
// accumulate / bias_grad; N % 8 == 0 and 16-B aligned C / bias / aux rows
// (-4 otherwise: use hvk_gemm).  ws_zero is ignored (every slice element is
// written before it is read).
HVK_API int hvk_gemm_splitk(int transA, int transB, int M, int N, int K,
                            const void* A, int lda, const void* B, int ldb,
                            void* C, int ldc, int out_f32, float alpha,
                            const float* bias, int act, const void* aux,
                            int ld_aux, int aux_act, int splits, float* ws,
                            int ws_zero, hipStream_t s) {
  (void)ws_zero;
  Epi e = make_epi(C, ldc, M, N, out_f32, 0, alpha, 0.f, bias, 1, act, aux,
                   ld_aux, aux_act);
  if (N % 8 || !e.fast_ok() || ((uintptr_t)ws & 15) || splits < 2) return -4;
  // the split count launch() derives (K per split rounded up to BK)
  int ks = (K + splits - 1) / splits;
  ks = (ks + BK - 1) / BK * BK;
  const int sp = (K + ks - 1) / ks;
  Epi w = make_epi(ws, N, M, N, 1, 0, 1.f, 0.f, nullptr, 0, 0, nullptr, 0, 0);
  w.slice = 1;
  w.grow = M;
  const hipError_t err = gemm_dispatch(transA, transB, M, N, K,
                                       (const uint16_t*)A, lda,
                                       (const uint16_t*)B, ldb, w, splits, -1,
                                       s);
  if (err != hipSuccess) return (int)err;
  const long long total = (long long)M * (N / 8);
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(splitk_finish_kernel, dim3((int)blocks), dim3(256), 0, s,
                     (const float*)ws, M, N, sp, e);
  return (int)launch_status(s);
}

