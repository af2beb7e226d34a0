// gemm_conv_fwd.hip - implicit-GEMM convolution forward on the gemm_core.h main loop
#include "gemm_core.h"

// Y[n][oh][ow][oc] = act(sum X*W + bias); X NHWC bf16, W [OC][KH][KW][C/g]
static int conv_fwd(const void* X, const void* Wt, const float* bias, void* Y,
                    int N, int H, int W, int C, int OC, int KH, int KW, int sy,
                    int sx, int pt, int pl, int OH, int OW, int groups,
                    int act, const Q8* q8, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  int M = N * OH * OW, K = KH * KW * g.Cg;
  ConvFwdA la{(const uint16_t*)X, g, M, K,
              (g.Cg % 8 == 0 && C % 8 == 0 && al16(X)) ? 1 : 0, 0};
  DenseK lb{(const uint16_t*)Wt, (long long)g.OCg * K, g.OCg, K, K,
            (K % 8 == 0 && al16(Wt)) ? 1 : 0};
  Epi e = make_epi(Y, OC, M, g.OCg, 0, 0, 1.f, 0.f, bias, 1, act, nullptr, 0, 0);
  e.gcol = g.OCg;
  if (q8) {
    if (!e.fast_ok() || g.OCg % 8 || (((uintptr_t)q8->q) & 7)) return -3;
    e.q8 = *q8;
  }
  return (int)launch<ConvFwdA, true, DenseK, true>(la, lb, e, M, g.OCg, K, 1,
                                                   groups, s);
}

HVK_API int hvk_conv_fwd(const void* X, const void* Wt, const float* bias,
                         void* Y, int N, int H, int W, int C, int OC, int KH,
                         int KW, int sy, int sx, int pt, int pl, int OH, int OW,
                         int groups, int act, hipStream_t s) {
  return conv_fwd(X, Wt, bias, Y, N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH,
                  OW, groups, act, nullptr, s);
}

// as hvk_conv_fwd, and the fp8 copy of Y for the fp8 layer reading it (the
// q8 arguments of hvk_conv_fwd_halo_q8)
HVK_API int hvk_conv_fwd_q8(const void* X, const void* Wt, const float* bias,
                            void* Y, int N, int H, int W, int C, int OC,
                            int KH, int KW, int sy, int sx, int pt, int pl,
                            int OH, int OW, int groups, int act, void* q8,
                            const float* q8_st, float* q8_shard,
                            float q8_fmax, int q8_fmt, int hist,
                            hipStream_t s) {
  const Q8 z{(uint8_t*)q8, q8_st, q8_shard, q8_fmax, q8_fmt, hist};
  return conv_fwd(X, Wt, bias, Y, N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH,
                  OW, groups, act, &z, s);
}

// Small-channel forward: Wp is [OC][KH][RUNP] (zero padded runs)
HVK_API int hvk_conv_fwd_run(const void* X, const void* Wp, const float* bias,
                             void* Y, int N, int H, int W, int C, int OC,
                             int KH, int KW, int sy, int sx, int pt, int pl,
                             int OH, int OW, int act, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, 1);
  RunGeom r = make_run(g);
  int M = N * OH * OW, K = KH * r.RUNP;
  ConvFwdRunA la{(const uint16_t*)X, g, r, M, K};
  DenseK lb{(const uint16_t*)Wp, 0, OC, K, K, al16(Wp) ? 1 : 0};
  Epi e = make_epi(Y, OC, M, OC, 0, 0, 1.f, 0.f, bias, 1, act, nullptr, 0, 0);
  return (int)launch<ConvFwdRunA, true, DenseK, true>(la, lb, e, M, OC, K, 1, 1,
                                                      s);
}

