// conv_geom.h - NHWC convolution geometry shared by the bf16 (gemm.hip) and
// fp8 (gemm_fp8.hip) implicit-GEMM kernels.  All index math in the loaders
// goes through FastDiv (one mul_hi + add + shift per division).
#pragma once
#include "hvk_common.h"

namespace hvk {

struct ConvGeom {
  int N, H, W, C, Cg;       // input NHWC, C total, Cg per group
  int OH, OW, OC, OCg;      // output
  int KH, KW, sy, sx, pt, pl;
  FastDiv fOW, fOHOW, fW, fHW, fCg, fOCg, fKW, fSy, fSx;
};

inline ConvGeom make_geom(int N, int H, int W, int C, int OC, int KH, int KW,
                          int sy, int sx, int pt, int pl, int OH, int OW,
                          int groups) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Cg = C / groups;
  g.OH = OH; g.OW = OW; g.OC = OC; g.OCg = OC / groups;
  g.KH = KH; g.KW = KW; g.sy = sy; g.sx = sx; g.pt = pt; g.pl = pl;
  g.fOW = make_fastdiv(OW); g.fOHOW = make_fastdiv(OH * OW);
  g.fW = make_fastdiv(W); g.fHW = make_fastdiv(H * W);
  g.fCg = make_fastdiv(g.Cg); g.fOCg = make_fastdiv(g.OCg);
  g.fKW = make_fastdiv(KW);
  g.fSy = make_fastdiv(sy);
  g.fSx = make_fastdiv(sx);
  return g;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md T1):
// consecutive logical workgroup ids land on one XCD (private L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace hvk
