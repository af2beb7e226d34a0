"""Same-process A/B of the conv weight-gradient kernels on the AlexNet (and
VGG-16) layer shapes: the halo kernel (csrc/kernels/wgrad_halo.hip) against
the 128-row / T4 GEMM loops (ops.set_halo_wgrad(False)), interleaved round
by round in ONE process on random operands (cdna_hip_programming.md §5.4
rules 24-25), reporting the median TF/s per setting.

    python tools/bench_wgrad_ab.py [alexnet_batch] [rounds] [vgg_batch]

Writes gpurun_out/bench_wgrad_ab.json."""
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


def case(N, H, W, C, OC, k, p, g, st=1):
    OH, OW = ops.conv_out_size(H, W, k, k, (st, st), (p, p, p, p))
    x = (torch.rand(N, H, W, C, device="cuda") * 2 - 1).to(BF)
    dy = (torch.rand(N, OH, OW, OC, device="cuda") * 2 - 1).to(BF)
    dw = torch.zeros(OC, k, k, C // g, device="cuda")
    db = torch.zeros(OC, device="cuda")
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    return fl, lambda: ops.conv_wgrad(x, dy, dw, (st, st), (p, p, p, p), g,
                                      dbias=db)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    VB = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cases = [("alex_conv1", (B, 227, 227, 3, 96, 11, 0, 1, 4)),
             ("alex_conv2", (B, 27, 27, 96, 256, 5, 2, 2)),
             ("alex_conv3", (B, 13, 13, 256, 384, 3, 1, 1)),
             ("alex_conv4", (B, 13, 13, 384, 384, 3, 1, 2)),
             ("alex_conv5", (B, 13, 13, 384, 256, 3, 1, 2))]
    if VB:
        cases += [("vgg_conv1_2", (VB // 4, 224, 224, 64, 64, 3, 1, 1)),
                  ("vgg_conv2_2", (VB // 2, 112, 112, 128, 128, 3, 1, 1)),
                  ("vgg_conv3_2", (VB, 56, 56, 256, 256, 3, 1, 1)),
                  ("vgg_conv4_2", (VB, 28, 28, 512, 512, 3, 1, 1)),
                  ("vgg_conv5_2", (VB, 14, 14, 512, 512, 3, 1, 1))]
    out = {}
    for name, shp in cases:
        fl, fn = case(*shp)
        res = {"halo": [], "gemm": []}
        for _ in range(rounds):
            for key, on in (("halo", True), ("gemm", False)):
                ops.set_halo_wgrad(on)
                res[key].append(fl / timeit(fn) / 1e12)
        ops.set_halo_wgrad(True)
        med = {k: statistics.median(v) for k, v in res.items()}
        out[name] = {"shape": shp, "tflops": med, "runs": res}
        print("%-12s halo %7.1f TF  gemm %7.1f TF  (%.2fx)" % (
            name, med["halo"], med["gemm"], med["halo"] / med["gemm"]),
            flush=True)
        del fn
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_wgrad_ab.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
