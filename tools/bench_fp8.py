"""FP8 vs bf16 kernel micro-benchmarks on square GEMMs and VGG-16 layer
shapes (random operands, one process, interleaved; cdna_hip_programming.md
§5.4 rules 24/25).  Writes gpurun_out/bench_fp8.json.

    python tools/bench_fp8.py [batch] [fp8 variant ...]

With a variant list the fp8 convolutions are timed once per
hvk_set_fp8_variant setting (A/B of the fp8 loops)."""
import json
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402
from veles_amd.ops import fp8  # noqa: E402

dev = "cuda"
VARS = [int(v) for v in sys.argv[2:]] or [-1]
BF = torch.bfloat16
res = {}


def timeit(fn, n=20, w=3):
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


def q(x, fmt=fp8.E4M3):
    s = fp8.Scaler(dev, fmt)
    return fp8.quantize(x, s), s


def gemm_case(name, M, N, K):
    a = torch.randn(M, K, device=dev).to(BF)
    b = torch.randn(N, K, device=dev).to(BF)
    a8, sa = q(a)
    b8, sb = q(b)
    out = torch.empty(M, N, device=dev, dtype=BF)
    t_b = timeit(lambda: ops.gemm(a, b, trans_b=True, out=out))
    t_8 = timeit(lambda: fp8.gemm(a8, sa, b8, sb, out=out))
    t_q = timeit(lambda: fp8.quantize(a, sa, out=a8))
    fl = 2.0 * M * N * K
    res[name] = {"bf16_TF": fl / t_b / 1e12, "fp8_TF": fl / t_8 / 1e12,
                 "quant_ms": t_q * 1e3}
    print(name, res[name], flush=True)


def conv_case(name, N, H, W, C, OC, k=3, p=1):
    x = torch.randn(N, H, W, C, device=dev).to(BF)
    w = (torch.randn(OC, k, k, C, device=dev) * 0.05).to(BF)
    b = torch.randn(OC, device=dev)
    dy = (torch.randn(N, H, W, OC, device=dev) * 1e-2).to(BF)
    pad = (p, p, p, p)
    x8, sx = q(x)
    w8, sw = q(w)
    d8, sd = q(dy, fp8.E5M2)
    wt8 = fp8.permute_for_dgrad(w8, 1)
    fl = 2.0 * N * H * W * OC * k * k * C
    r = {
        "fwd_bf16_TF": fl / timeit(lambda: ops.conv_fwd(
            x, w, b, (1, 1), pad, 1, 3)) / 1e12,
        "dgrad_bf16_TF": fl / timeit(lambda: ops.conv_dgrad(
            dy, w, (N, H, W, C), (1, 1), pad, 1)) / 1e12,
    }
    lib = ops._lib.lib()
    for v in VARS:
        sfx = "" if VARS == [-1] else "_v%d" % v
        lib.hvk_set_fp8_variant(v)
        r["fwd_fp8_TF" + sfx] = fl / timeit(lambda: fp8.conv_fwd(
            x8, sx, w8, sw, b, (1, 1), pad, 1, 3)) / 1e12
        r["dgrad_fp8_TF" + sfx] = fl / timeit(lambda: fp8.conv_dgrad(
            d8, sd, w8, sw, (N, H, W, C), (1, 1), pad, 1, wt8=wt8)) / 1e12
    lib.hvk_set_fp8_variant(-1)
    res[name] = r
    print(name, r, flush=True)


gemm_case("gemm_4096", 4096, 4096, 4096)
gemm_case("gemm_8192", 8192, 8192, 8192)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
gemm_case("vgg_fc6_fwd", B, 4096, 25088)
conv_case("vgg_conv1_2", B, 224, 224, 64, 64)
conv_case("vgg_conv2_2", B, 112, 112, 128, 128)
conv_case("vgg_conv3_2", B, 56, 56, 256, 256)
conv_case("vgg_conv4_2", B, 28, 28, 512, 512)
conv_case("vgg_conv5_2", B, 14, 14, 512, 512)
json.dump(res, open("gpurun_out/bench_fp8.json", "w"), indent=1)
