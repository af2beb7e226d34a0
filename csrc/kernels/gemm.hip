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

// Split-K finishing pass: C = epilogue(ws), ws the f32 sum of the K splits
// (N % 8 == 0 and Epi::fast_ok(): one 8-column chunk per thread)
__global__ void splitk_finish_kernel(float* __restrict__ ws, int M, int N,
                                     Epi e, int clear) {
  const int CH = N >> 3;
  const long long total = (long long)M * CH;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       q < total; q += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(q / CH), c8 = (int)(q - (long long)m * CH) * 8;
    float4* src = (float4*)(ws + (long long)m * N + c8);
    const float4 lo = src[0], hi = src[1];
    if (clear) {  // leave the workspace zeroed for the next split-K GEMM
      src[0] = make_float4(0.f, 0.f, 0.f, 0.f);
      src[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    e.store8_fast(0, m, c8, v);
  }
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
  const int oc = bias_grad ? N : -1;
  const uint16_t* a = (const uint16_t*)A;
  const uint16_t* b = (const uint16_t*)B;
  int va = al16(a) && (lda % 8 == 0), vb = al16(b) && (ldb % 8 == 0);
  hipError_t err;
  if (!transA && transB) {
    DenseK la{a, 0, M, K, lda, va};
    DenseK lb{b, 0, N, K, ldb, vb};
    err = launch<DenseK, true, DenseK, true>(la, lb, e, M, N, K, splits, 1, s);
  } else if (!transA && !transB) {
    DenseK la{a, 0, M, K, lda, va};
    DenseMN lb{b, 0, N, K, ldb, vb, oc};
    err = launch<DenseK, true, DenseMN, false>(la, lb, e, M, Nk, K, splits, 1, s);
  } else if (transA && !transB) {
    DenseMN la{a, 0, M, K, lda, va, -1};
    DenseMN lb{b, 0, N, K, ldb, vb, oc};
    err = launch<DenseMN, false, DenseMN, false>(la, lb, e, M, Nk, K, splits, 1, s);
  } else {
    DenseMN la{a, 0, M, K, lda, va, -1};
    DenseK lb{b, 0, N, K, ldb, vb};
    err = launch<DenseMN, false, DenseK, true>(la, lb, e, M, N, K, splits, 1, s);
  }
  return (int)err;
}

// Split-K GEMM for shapes with too few output tiles to fill 256 CUs (the FC
// layers at batch 512: fc6 forward is 4 x 32 tiles of 128 x 128): the K range
// is split `splits` ways, the partial products are summed by f32 atomics into
// the workspace ws[M][N] (zeroed here), then one pass applies alpha, the
// per-column bias, the activation and the aux derivative and casts to C.
// Same arguments as hvk_gemm minus beta / accumulate / bias_grad; N % 8 == 0
// and 16-B aligned C / bias / aux rows (-4 otherwise: use hvk_gemm).
// ws_zero = 1: ws is all zeros on entry and is left all zeros (the finishing
// pass clears what it read) - no memset launch per GEMM.
HVK_API int hvk_gemm_splitk(int transA, int transB, int M, int N, int K,
                            const void* A, int lda, const void* B, int ldb,
                            void* C, int ldc, int out_f32, float alpha,
                            const float* bias, int act, const void* aux,
                            int ld_aux, int aux_act, int splits, float* ws,
                            int ws_zero, hipStream_t s) {
  Epi e = make_epi(C, ldc, M, N, out_f32, 0, alpha, 0.f, bias, 1, act, aux,
                   ld_aux, aux_act);
  if (N % 8 || !e.fast_ok() || ((uintptr_t)ws & 15) || splits < 2) return -4;
  if (!ws_zero) {
    hipError_t err = hipMemsetAsync(ws, 0, (size_t)M * N * sizeof(float), s);
    if (err != hipSuccess) return (int)err;
  }
  const int rc = hvk_gemm(transA, transB, M, N, K, A, lda, B, ldb, ws, N, 1,
                          1, 1.f, 0.f, nullptr, 0, 0, nullptr, 0, 0, splits,
                          nullptr, s);
  if (rc) return rc;
  const long long total = (long long)M * (N / 8);
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(splitk_finish_kernel, dim3((int)blocks), dim3(256), 0, s,
                     ws, M, N, e, ws_zero);
  return (int)launch_status(s);
}

