// gemm_conv_dgrad.hip - implicit-GEMM convolution backward-data on the gemm_core.h main loop
#include "gemm_core.h"

// dgrad with the weights pre-permuted to Wt[g][c][kh][kw][oc] (k = (kh,kw,oc)
// fastest): the B operand is a dense K-major matrix [Cg][K] per group -- full
// lines through the LDS-DMA path, ds_read_b128 fragments, and a 64-wide B
// stage of 8 KiB (3 blocks per CU for Cg <= 64).
HVK_API int hvk_conv_dgrad_t(const void* dY, const void* Wt, void* dX, int N,
                             int H, int W, int C, int OC, int KH, int KW,
                             int sy, int sx, int pt, int pl, int OH, int OW,
                             int groups, const void* aux, int aux_act,
                             hipStream_t s) {
  ConvGeom g = make_geom(N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups);
  int M = N * H * W, K = KH * KW * g.OCg;
  const int vec = (g.OCg % 8 == 0 && OC % 8 == 0 && al16(dY)) ? 1 : 0;
  ConvDgradA la{(const uint16_t*)dY, g, M, K, vec, 0};
  DenseK lb{(const uint16_t*)Wt, (long long)K * g.Cg, g.Cg, K, K,
            (K % 8 == 0 && al16(Wt)) ? 1 : 0};
  Epi e = make_epi(dX, C, M, g.Cg, 0, 0, 1.f, 0.f, nullptr, 0, 0, aux, C, aux_act);
  e.gcol = g.Cg;
  if (!vec) {
    ConvDgradAS ls;
    static_cast<ConvDgradA&>(ls) = la;
    return (int)launch<ConvDgradAS, true, DenseK, true>(ls, lb, e, M, g.Cg,
                                                        K, 1, groups, s);
  }
  if (sy != 1 || sx != 1 || KH > 32 || KW > 32) {
    ConvDgradAStr ls;
    static_cast<ConvDgradA&>(ls) = la;
    return (int)launch<ConvDgradAStr, true, DenseK, true>(ls, lb, e, M, g.Cg,
                                                          K, 1, groups, s);
  }
  return (int)launch<ConvDgradA, true, DenseK, true>(la, lb, e, M, g.Cg, K,
                                                     1, groups, s);
}

