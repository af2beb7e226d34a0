"""Same-process A/B of the fp8 conv weight gradient on the VGG-16 layer
shapes: the fp8 halo kernel (wgrad_halo.hip wgrad_halo8_kernel) against
wgrad_fp8.hip (ops.set_halo_wgrad(False)), interleaved round by round in ONE
process on random operands, median TF/s per setting (MFMA work counted at
the logical 2 N OH OW OC KH KW C).

    python tools/bench_wgrad8_ab.py [vgg_batch] [rounds]

Writes gpurun_out/bench_wgrad8_ab.json."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402
from veles_amd.ops import fp8  # noqa: E402

DEV = "cuda"


def timeit(fn, n=6, w=2):
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


def case(N, H, W, C, OC):
    sx, sd = fp8.Scaler(DEV, fp8.E4M3), fp8.Scaler(DEV, fp8.E5M2)
    x8 = fp8.quantize((torch.randn(N, H, W, C, device=DEV)).to(
        torch.bfloat16), sx)
    d8 = fp8.quantize((torch.randn(N, H, W, OC, device=DEV) * 1e-2).to(
        torch.bfloat16), sd)
    dw = torch.zeros(OC, 3, 3, C, device=DEV)
    db = torch.zeros(OC, device=DEV)
    fl = 2.0 * N * H * W * OC * 9 * C
    return fl, lambda: fp8.conv_wgrad(x8, sx, d8, sd, dw, (1, 1),
                                      (1, 1, 1, 1), 1, dbias=db)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cases = [("vgg_conv1_2", (B, 224, 224, 64, 64)),
             ("vgg_conv2_1", (B, 112, 112, 64, 128)),
             ("vgg_conv2_2", (B, 112, 112, 128, 128)),
             ("vgg_conv3_2", (B, 56, 56, 256, 256)),
             ("vgg_conv4_2", (B, 28, 28, 512, 512)),
             ("vgg_conv5_2", (B, 14, 14, 512, 512))]
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
    with open("gpurun_out/bench_wgrad8_ab.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
