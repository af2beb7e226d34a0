// gemm_conv_fwd.hip - implicit-GEMM convolution forward on the gemm_core.h main loop
#include "gemm_core.h"

// Y[n][oh][ow][oc] = act(sum X*W + bias); X NHWC bf16, W [OC][KH][KW][C/g]
HVK_API int hvk_conv_fwd(const void* X, const void* Wt, const float* bias,
                         void* Y, int N, int H, int W, int C, int OC, int KH,
                         int KW, int sy, int sx, int pt, int pl, int OH, int OW,
                         int groups, int act, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  int M = N * OH * OW, K = KH * KW * g.Cg;
  ConvFwdA la{(const uint16_t*)X, g, M, K,
              (g.Cg % 8 == 0 && C % 8 == 0 && al16(X)) ? 1 : 0, 0};
  DenseK lb{(const uint16_t*)Wt, (long long)g.OCg * K, g.OCg, K, K,
            (K % 8 == 0 && al16(Wt)) ? 1 : 0};
  Epi e = make_epi(Y, OC, M, g.OCg, 0, 0, 1.f, 0.f, bias, 1, act, nullptr, 0, 0);
  e.gcol = g.OCg;
  return (int)launch<ConvFwdA, true, DenseK, true>(la, lb, e, M, g.OCg, K, 1,
                                                   groups, s);
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

