// hvk_api.h - C ABI of the veles_amd HIP kernel library (libhvk.so), used
// by the Python ops layer (ctypes) and by the native runtime (csrc/runtime).
#pragma once
#include <hip/hip_runtime.h>

extern "C" {
int hvk_gemm(int transA, int transB, int M, int N, int K, const void* A,
             int lda, const void* B, int ldb, void* C, int ldc, int out_f32,
             int atomic, float alpha, float beta, const float* bias,
             int bias_mode, int act, const void* aux, int ld_aux, int aux_act,
             int splits, float* bias_grad, hipStream_t s);
int hvk_gemm_splitk(int transA, int transB, int M, int N, int K,
                    const void* A, int lda, const void* B, int ldb, void* C,
                    int ldc, int out_f32, float alpha, const float* bias,
                    int act, const void* aux, int ld_aux, int aux_act,
                    int splits, float* ws, int ws_zero, hipStream_t s);
int hvk_conv_fwd(const void* X, const void* W, const float* bias, void* Y,
                 int N, int H, int Wd, int C, int OC, int KH, int KW, int sy,
                 int sx, int pt, int pl, int OH, int OW, int groups, int act,
                 hipStream_t s);
int hvk_conv_fwd_run(const void* X, const void* Wp, const float* bias, void* Y,
                     int N, int H, int Wd, int C, int OC, int KH, int KW,
                     int sy, int sx, int pt, int pl, int OH, int OW, int act,
                     hipStream_t s);
int hvk_pool_fwd(const void* x, void* y, int* argmax, int N, int H, int W,
                 int C, int OH, int OW, int ky, int kx, int sy, int sx, int pt,
                 int pl, int mode, hipStream_t s);
int hvk_lrn_fwd(const void* x, void* y, long long P, int C, int n, float alpha,
                float beta, float k, hipStream_t s);
int hvk_act_fwd(const void* x, int xdt, void* y, int ydt, long long n, int act,
                hipStream_t s);
int hvk_softmax_ce(const void* logits, int in_dt, int B, int C,
                   const int* labels, float scale, void* err, int err_dt,
                   float* probs, int* max_idx, float* metrics, int* confusion,
                   hipStream_t s);
int hvk_cast(const void* in, int idt, void* out, int odt, long long n,
             float scale, hipStream_t s);
}

enum { HVK_F32 = 0, HVK_BF16 = 1, HVK_U8 = 2, HVK_I32 = 3 };
