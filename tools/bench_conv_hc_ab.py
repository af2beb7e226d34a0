"""Same-process A/B of the channel-chunked halo conv kernels (conv_hc.hip)
against the kernels they replace (ops.set_conv_hc(False): T4 / 256x256
ping-pong / 128-row implicit GEMM / conv_halo), interleaved round by round
in ONE process on random operands; median TF/s at the logical
2 N OH OW OC KH KW C/g FLOPs.  Extra settings "hcV" force conv_hc.hip
configuration V.

    python tools/bench_conv_hc_ab.py [alexnet_batch] [rounds] [vgg_batch]
                                     [variants, e.g. 2,3]

Writes gpurun_out/bench_conv_hc_ab.json."""
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
    variants = [int(v) for v in sys.argv[4].split(",")] \
        if len(sys.argv) > 4 and sys.argv[4] else []
    cases = [("conv1_fwd", ("fwd", B, 227, 227, 3, 96, 11, 4, 0, 1)),
             ("conv2_fwd", ("fwd", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv3_fwd", ("fwd", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_fwd", ("fwd", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_fwd", ("fwd", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv2_dgrad", ("dgrad", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv3_dgrad", ("dgrad", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_dgrad", ("dgrad", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_dgrad", ("dgrad", B, 13, 13, 384, 256, 3, 1, 1, 2))]
    if VB:
        cases += [("vgg_conv1_2_fwd", ("fwd", VB // 4, 224, 224, 64, 64, 3,
                                       1, 1, 1)),
                  ("vgg_conv1_2_dgrad", ("dgrad", VB // 4, 224, 224, 64, 64,
                                         3, 1, 1, 1)),
                  ("vgg_conv4_2_fwd", ("fwd", VB, 28, 28, 512, 512, 3, 1, 1,
                                       1)),
                  ("vgg_conv4_2_dgrad", ("dgrad", VB, 28, 28, 512, 512, 3, 1,
                                         1, 1)),
                  ("vgg_conv2_2_fwd", ("fwd", VB // 2, 112, 112, 128, 128, 3,
                                       1, 1, 1)),
                  ("vgg_conv3_2_fwd", ("fwd", VB, 56, 56, 256, 256, 3, 1, 1,
                                       1)),
                  ("vgg_conv3_2_dgrad", ("dgrad", VB, 56, 56, 256, 256, 3, 1,
                                         1, 1))]
    # hc: the automatic policy (conv_hc32 where it applies); hc16: the same
    # with the 32x32x16 configurations off; base: no halo conv at all
    settings = [("hc", True, -2, True), ("hc16", True, -2, False),
                ("base", False, -2, True)] + \
        [("hc%d" % v, True, v, True) for v in variants]
    out = {}
    for name, shp in cases:
        fl, fn = case(*shp)
        res = {k: [] for k, _, _, _ in settings}
        taken = {}
        for _ in range(rounds):
            for key, on, var, m32 in settings:
                ops.set_conv_hc(on, var)
                ops.set_conv_hc32(m32)
                res[key].append(fl / timeit(fn) / 1e12)
                taken[key] = ops.conv_hc_last_variant() if on else 0
        ops.set_conv_hc(True, -2)
        ops.set_conv_hc32(True)
        med = {k: statistics.median(v) for k, v in res.items()}
        out[name] = {"shape": shp, "tflops": med, "runs": res,
                     "variant": taken}
        print("%-18s " % name + "  ".join(
            "%s %7.1f TF" % (k, med[k]) for k, _, _, _ in settings) +
            "  (hc/hc16 %.2fx, hc/base %.2fx; hc var %d)" % (
                med["hc"] / med["hc16"], med["hc"] / med["base"],
                taken["hc"]), flush=True)
        del fn
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bench_conv_hc_ab.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
