"""Conv implicit-GEMM vs the plain dense GEMM of the same M/N/K (per group):
does the implicit-GEMM address arithmetic cost MFMA rate?"""
import statistics, sys
import torch
sys.path.insert(0, ".")
import veles_amd.ops as ops
sys.path.insert(0, "tools")
from bench_gemm_ab import timeit, gemm, conv
B = 512
layers = {"conv2": (B, 27, 27, 96, 256, 5, 1, 2, 2),
          "conv3": (B, 13, 13, 256, 384, 3, 1, 1, 1),
          "conv4": (B, 13, 13, 384, 384, 3, 1, 1, 2),
          "conv5": (B, 13, 13, 384, 256, 3, 1, 1, 2)}
for name, (N, H, W, C, OC, k, s, p, g) in layers.items():
    OH = (H + 2 * p - k) // s + 1
    M = N * OH * OH
    Cg, OCg = C // g, OC // g
    eq = {"fwd": (M, OCg, k * k * Cg, False, True),
          "dgrad": (N * H * W, Cg, k * k * OCg, False, True),
          "wgrad": (OCg, k * k * Cg, M, True, False)}
    for kind in ("fwd", "dgrad", "wgrad"):
        fl, fc = conv(kind, N, H, W, C, OC, k, s, p, g)
        Mx, Nx, Kx, ta, tb = eq[kind]
        fl2, fp = gemm(Mx, Nx, Kx, ta, tb)
        tc, tp = [], []
        for _ in range(5):
            tc.append(timeit(fc)); tp.append(timeit(fp))
        print("%s_%s conv=%.0fTF plain(M=%d,N=%d,K=%d)=%.0fTF" % (
            name, kind, fl / statistics.median(tc) / 1e12, Mx, Nx, Kx,
            fl2 / statistics.median(tp) / 1e12), flush=True)
