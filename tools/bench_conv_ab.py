"""Same-process A/B of the weight-stationary conv kernels (conv_ws.hip)
against the implicit-GEMM / halo paths they replace (ops.set_conv_ws(False)),
interleaved round by round in ONE process on random operands; median TF/s
at the logical 2 N OH OW OC KH KW C/g FLOPs.

    python tools/bench_conv_ab.py [alexnet_batch] [rounds] [vgg_batch]

Writes gpurun_out/bench_conv_ab.json."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

BF = torch.bfloat16


def timeit(fn, n=8, w=2):
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


def case(kind, N, H, W, C, OC, k, st, p, g):
    OH, OW = ops.conv_out_size(H, W, k, k, (st, st), (p, p, p, p))
    x = (torch.rand(N, H, W, C, device="cuda") * 2 - 1).to(BF)
    w = ((torch.rand(OC, k, k, C // g, device="cuda") * 2 - 1) * 0.05).to(BF)
    b = torch.randn(OC, device="cuda")
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    if kind == "fwd":
        y = torch.empty(N, OH, OW, OC, device="cuda", dtype=BF)
        return fl, lambda: ops.conv_fwd(x, w, b, (st, st), (p, p, p, p), g,
                                        "str", out=y)
    dy = (torch.rand(N, OH, OW, OC, device="cuda") * 2 - 1).to(BF)
    dx = torch.empty(N, H, W, C, device="cuda", dtype=BF)
    return fl, lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (st, st),
                                      (p, p, p, p), g, aux=x, aux_act="str",
                                      out=dx)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    VB = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cases = [("alex_conv1_fwd", ("fwd", B, 227, 227, 3, 96, 11, 4, 0, 1)),
             ("alex_conv2_fwd", ("fwd", B, 27, 27, 96, 256, 5, 1, 2, 2))]
    if VB:
        cases += [("vgg_conv1_2_fwd", ("fwd", VB, 224, 224, 64, 64, 3, 1, 1,
                                       1)),
                  ("vgg_conv1_2_dgrad", ("dgrad", VB, 224, 224, 64, 64, 3, 1,
                                         1, 1))]
    out = {}
    for name, shp in cases:
        fl, fn = case(*shp)
        res = {"ws": [], "gemm": []}
        for _ in range(rounds):
            for key, on in (("ws", True), ("gemm", False)):
                ops.set_conv_ws(on)
                res[key].append(fl / timeit(fn) / 1e12)
        ops.set_conv_ws(False)
        med = {k: statistics.median(v) for k, v in res.items()}
        out[name] = {"shape": shp, "tflops": med, "runs": res}
        print("%-18s ws %7.1f TF  gemm %7.1f TF  (%.2fx)" % (
            name, med["ws"], med["gemm"], med["ws"] / med["gemm"]),
            flush=True)
        del fn
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_conv_ab.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
