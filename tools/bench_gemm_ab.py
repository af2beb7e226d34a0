"""A/B harness for bf16 GEMM main-loop variants of libhvk.so on the
AlexNet / VGG layer shapes, interleaved in ONE process (cdna_hip_programming.md
§5.4 rule 24) on random operands (rule 25).  A variant build exports
``hvk_set_gemm_variant(int)``; without it only the shipped loop is timed.
The round-2 deep-ring and ping-pong experiments ran through this script
(profiles/gemm_experiments_r2.md).

    python tools/bench_gemm_ab.py [batch] [rounds]

Prints one line per case: median TF of every setting over the rounds, and
writes gpurun_out/bench_gemm_ab.json."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

dev = "cuda"
BF = torch.bfloat16
SETTINGS = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3
                             else "0,1").split(",")]


def select(v):
    fn = getattr(ops._lib.lib(), "hvk_set_gemm_variant", None)
    if fn is not None:
        fn(int(v))


def timeit(fn, n=10, w=2):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def gemm(M, N, K, ta=False, tb=True):
    a = (torch.rand(K, M, device=dev) * 2 - 1).to(BF) if ta else \
        (torch.rand(M, K, device=dev) * 2 - 1).to(BF)
    b = (torch.rand(N, K, device=dev) * 2 - 1).to(BF) if tb else \
        (torch.rand(K, N, device=dev) * 2 - 1).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    return 2.0 * M * N * K, lambda: ops.gemm(a, b, trans_a=ta, trans_b=tb,
                                             out=out)


def conv(kind, N, H, W, C, OC, k, s, p, g):
    x = (torch.rand(N, H, W, C, device=dev) * 2 - 1).to(BF)
    w = ((torch.rand(OC, k, k, C // g, device=dev) * 2 - 1) * 0.05).to(BF)
    b = torch.randn(OC, device=dev)
    OH, OW = ops.conv_out_size(H, W, k, k, (s, s), (p, p, p, p))
    dy = (torch.rand(N, OH, OW, OC, device=dev) * 2 - 1).to(BF)
    dw = torch.zeros(OC, k, k, C // g, device=dev)
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    if kind == "fwd":
        return fl, lambda: ops.conv_fwd(x, w, b, (s, s), (p, p, p, p), g, 3)
    if kind == "dgrad":
        return fl, lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (s, s),
                                          (p, p, p, p), g)
    return fl, lambda: ops.conv_wgrad(x, dy, dw, (s, s), (p, p, p, p), g)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cases = [("gemm_4096", lambda: gemm(4096, 4096, 4096)),
             ("gemm_8192", lambda: gemm(8192, 8192, 8192)),
             ("gemm_8192_nn", lambda: gemm(8192, 8192, 8192, tb=False)),
             ("fc6_fwd", lambda: gemm(B, 4096, 9216)),
             ("fc6_dgrad", lambda: gemm(B, 9216, 4096, tb=False)),
             ("fc6_wgrad", lambda: gemm(4096, 9216, B, ta=True, tb=False))]
    # conv1 after space-to-depth (57 x 57 x 48 -> 55 x 55 x 96, 3 x 3)
    layers = {"conv1s2d": (B, 57, 57, 48, 96, 3, 1, 0, 1),
              "conv2": (B, 27, 27, 96, 256, 5, 1, 2, 2),
              "conv3": (B, 13, 13, 256, 384, 3, 1, 1, 1),
              "conv4": (B, 13, 13, 384, 384, 3, 1, 1, 2),
              "conv5": (B, 13, 13, 384, 256, 3, 1, 1, 2),
              "vgg3_2": (64, 56, 56, 256, 256, 3, 1, 1, 1)}
    for name, geo in layers.items():
        for kind in ("fwd", "dgrad", "wgrad"):
            cases.append(("%s_%s" % (name, kind),
                          lambda kind=kind, geo=geo: conv(kind, *geo)))
    res = {}
    for name, make in cases:
        fl, fn = make()
        settings = SETTINGS if getattr(ops._lib.lib(), "hvk_set_gemm_variant",
                                       None) else SETTINGS[:1]
        ts = {r: [] for r in settings}
        for _ in range(rounds):
            for r in settings:
                select(r)
                ts[r].append(timeit(fn))
        med = {r: fl / statistics.median(v) / 1e12 for r, v in ts.items()}
        res[name] = {"TF": {str(r): round(v, 1) for r, v in med.items()},
                     "best_ms": {str(r): round(min(v) * 1e3, 4)
                                 for r, v in ts.items()}}
        print(name, " ".join("v%d=%.0fTF" % (r, v)
                             for r, v in med.items()), flush=True)
        del fn
        torch.cuda.empty_cache()
    json.dump(res, open("gpurun_out/bench_gemm_ab.json", "w"), indent=1)


if __name__ == "__main__":
    main()
