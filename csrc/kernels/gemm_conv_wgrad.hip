// gemm_conv_wgrad.hip - implicit-GEMM convolution weight gradient on the gemm_core.h main loop
#include "gemm_core.h"

// dW[oc][kh][kw][c] (+)= sum_p dY[p][oc] * im2col(X)[p][kk]  (f32, atomics)
HVK_API int hvk_conv_wgrad(const void* X, const void* dY, float* dW, int N,
                           int H, int W, int C, int OC, int KH, int KW, int sy,
                           int sx, int pt, int pl, int OH, int OW, int groups,
                           int splits, float* dbias, hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  int P = N * OH * OW, KK = KH * KW * g.Cg;
  DenseMN la{(const uint16_t*)dY, (long long)g.OCg, g.OCg, P, OC,
             (OC % 8 == 0 && g.OCg % 8 == 0 && al16(dY)) ? 1 : 0, -1};
  ConvWgradB lb{(const uint16_t*)X, g, P, KK,
                (g.Cg % 8 == 0 && C % 8 == 0 && al16(X)) ? 1 : 0, 0,
                dbias ? 1 : 0};
  const int Nk = dbias ? KK + 1 : KK;
  Epi e = make_epi(dW, KK, g.OCg, Nk, 1, 1, 1.f, 0.f, nullptr, 0, 0, nullptr, 0, 0);
  e.grow = g.OCg;
  if (dbias) {
    e.ones_col = KK;
    e.bias_grad = dbias;
  }
  if (OH * OW < BK) {
    ConvWgradBGen lg;
    static_cast<ConvWgradB&>(lg) = lb;
    return (int)launch<DenseMN, false, ConvWgradBGen, false>(
        la, lg, e, g.OCg, Nk, P, splits, groups, s);
  }
  return (int)launch<DenseMN, false, ConvWgradB, false>(la, lb, e, g.OCg, Nk, P,
                                                        splits, groups, s);
}

// Small-channel weight gradient into dW [OC][KH][KW][C] (+ fused bias grad)
HVK_API int hvk_conv_wgrad_run(const void* X, const void* dY, float* dW,
                               float* dbias, int N, int H, int W, int C,
                               int OC, int KH, int KW, int sy, int sx, int pt,
                               int pl, int OH, int OW, int splits,
                               hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, 1);
  RunGeom r = make_run(g);
  int P = N * OH * OW, KKp = KH * r.RUNP;
  DenseMN la{(const uint16_t*)dY, 0, OC, P, OC,
             (OC % 8 == 0 && al16(dY)) ? 1 : 0, -1};
  ConvWgradRunB lb{(const uint16_t*)X, g, r, P, KKp, dbias ? 1 : 0};
  const int Nk = dbias ? KKp + 1 : KKp;
  Epi e = make_epi(dW, KH * r.RUN, OC, Nk, 1, 1, 1.f, 0.f, nullptr, 0, 0,
                   nullptr, 0, 0);
  e.run_in = r.RUNP;
  e.run_out = r.RUN;
  if (dbias) {
    e.ones_col = KKp;
    e.bias_grad = dbias;
  }
  return (int)launch<DenseMN, false, ConvWgradRunB, false>(la, lb, e, OC, Nk, P,
                                                           splits, 1, s);
}
