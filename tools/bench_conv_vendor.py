"""Per-layer bar against the vendor stack: this repo's conv kernels
(ops.conv_fwd / conv_dgrad / conv_wgrad, the default policy) against MIOpen
through torch (F.conv2d and aten.convolution_backward, bf16, channels-last,
cudnn.benchmark on so MIOpen searches its solvers), for every AlexNet and
VGG-16 convolution, on the same random operands, interleaved round by round
in ONE process.  TF/s at the logical 2 N OH OW OC KH KW C/g FLOPs (AlexNet
conv1 counted with its 11x11 taps, not the space-to-depth 3x3).

    python tools/bench_conv_vendor.py [alexnet_batch] [vgg_batch] [rounds]
    python tools/bench_conv_vendor.py --probe [alexnet_batch]

``--probe`` runs only our kernels, three calls per layer and direction, for
rocprofv3 --pmc passes (tools/gpu_pmc_kernels.sh).  Writes
gpurun_out/bench_conv_vendor.json."""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

BF = torch.bfloat16

ALEX = [("conv1", 227, 227, 3, 96, 11, 4, 0, 1),
        ("conv2", 27, 27, 96, 256, 5, 1, 2, 2),
        ("conv3", 13, 13, 256, 384, 3, 1, 1, 1),
        ("conv4", 13, 13, 384, 384, 3, 1, 1, 2),
        ("conv5", 13, 13, 384, 256, 3, 1, 1, 2)]
# VGG-16: (name, H, C, OC, batch divisor) - the batch shrinks with the
# image so each layer stays a few GB
VGG = [("vgg1_1", 224, 3, 64, 4), ("vgg1_2", 224, 64, 64, 4),
       ("vgg2_1", 112, 64, 128, 2), ("vgg2_2", 112, 128, 128, 2),
       ("vgg3_1", 56, 128, 256, 1), ("vgg3_2", 56, 256, 256, 1),
       ("vgg4_1", 28, 256, 512, 1), ("vgg4_2", 28, 512, 512, 1),
       ("vgg5_2", 14, 512, 512, 1)]


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


def layer(N, H, W, C, OC, k, st, p, g):
    """The callables of one layer: ours and MIOpen's per direction."""
    OH, OW = ops.conv_out_size(H, W, k, k, (st, st), (p, p, p, p))
    x = (torch.rand(N, H, W, C, device="cuda") * 2 - 1).to(BF)
    w = ((torch.rand(OC, k, k, C // g, device="cuda") * 2 - 1) * 0.05).to(BF)
    b = torch.randn(OC, device="cuda")
    dy = (torch.rand(N, OH, OW, OC, device="cuda") * 2 - 1).to(BF)
    y = torch.empty(N, OH, OW, OC, device="cuda", dtype=BF)
    dx = torch.empty(N, H, W, C, device="cuda", dtype=BF)
    dw = torch.zeros(OC, k, k, C // g, device="cuda", dtype=torch.float32)
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    pad = (p, p, p, p)
    xo = x
    s2 = ops.s2d_factor(C, g, (st, st), k, k)
    if s2:   # conv1: the loader-made space-to-depth image, as in the bench
        xo = ops.S2DImage(ops.space_to_depth(x, s2, k, k, pad), s2,
                          (N, H, W, C))
    ours = {
        "fwd": lambda: ops.conv_fwd(xo, w, b, (st, st), pad, g, "str", out=y),
        "dgrad": lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (st, st), pad,
                                        g, out=dx),
        "wgrad": lambda: ops.conv_wgrad(xo, dy, dw, (st, st), pad, g),
    }
    # torch views of the same bytes: NCHW shape, channels-last strides
    xc, wc = x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2)
    dyc = dy.permute(0, 3, 1, 2)
    bb = b.to(BF)
    cb = torch.ops.aten.convolution_backward
    args = ([st, st], [p, p], [1, 1], False, [0, 0], g)
    vendor = {
        "fwd": lambda: F.conv2d(xc, wc, bb, st, p, 1, g),
        "dgrad": lambda: cb(dyc, xc, wc, None, *args, [True, False, False]),
        "wgrad": lambda: cb(dyc, xc, wc, None, *args, [False, True, False]),
    }
    if C < 16:   # first layers: no data gradient in a training step
        del ours["dgrad"], vendor["dgrad"]
    return fl, ours, vendor


def shapes(B, VB):
    out = [(n, (B, H, W, C, OC, k, s, p, g)) for n, H, W, C, OC, k, s, p, g
           in ALEX]
    if VB:
        out += [(n, (VB // d, H, H, C, OC, 3, 1, 1, 1))
                for n, H, C, OC, d in VGG]
    return out


def main():
    if sys.argv[1:2] == ["--probe"]:
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
        for name, shp in shapes(B, 0):
            _, ours, _ = layer(*shp)
            for _ in range(3):
                for fn in ours.values():
                    fn()
            torch.cuda.synchronize()
            del ours
            torch.cuda.empty_cache()
        return
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    VB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.backends.cudnn.benchmark = True
    res = {}
    os.makedirs("gpurun_out", exist_ok=True)
    for name, shp in shapes(B, VB):
        fl, ours, vendor = layer(*shp)
        for d in ours:
            t = {"ours": [], "miopen": []}
            for _ in range(rounds):
                t["ours"].append(fl / timeit(ours[d]) / 1e12)
                t["miopen"].append(fl / timeit(vendor[d]) / 1e12)
            med = {k: statistics.median(v) for k, v in t.items()}
            res["%s_%s" % (name, d)] = {"shape": shp, "tflops": med,
                                        "runs": t}
            print("%-8s %-6s ours %7.1f TF  miopen %7.1f TF  (%.2fx)" % (
                name, d, med["ours"], med["miopen"],
                med["ours"] / med["miopen"]), flush=True)
            with open("gpurun_out/bench_conv_vendor.json", "w") as f:
                json.dump(res, f, indent=1)
        del ours, vendor
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
