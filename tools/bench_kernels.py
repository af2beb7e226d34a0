"""Kernel micro-benchmarks: hand-written HIP kernels vs the vendor libraries
(hipBLASLt GEMM / MIOpen conv through PyTorch) on the AlexNet layer shapes.

Writes gpurun_out/bench_kernels.json.  Random operands (cdna_hip_programming
§5.4 rule 25), interleaved timing in one process (rule 24).
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

dev = "cuda"
BF = torch.bfloat16
res = {}
TAG = os.environ.get("HVK_BENCH_TAG", "")


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


def gemm_case(name, M, N, K, ta=False, tb=True):
    a = torch.randn(K, M, device=dev).to(BF) if ta else torch.randn(M, K, device=dev).to(BF)
    b = torch.randn(N, K, device=dev).to(BF) if tb else torch.randn(K, N, device=dev).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    t_h = timeit(lambda: ops.gemm(a, b, trans_a=ta, trans_b=tb, out=out))
    A = a.t() if ta else a
    B = b.t() if tb else b
    t_t = timeit(lambda: torch.matmul(A, B))
    fl = 2.0 * M * N * K
    res[name] = {"hvk_TF": fl / t_h / 1e12, "torch_TF": fl / t_t / 1e12,
                 "hvk_ms": t_h * 1e3, "torch_ms": t_t * 1e3}
    print(name, res[name], flush=True)


def conv_case(name, N, H, W, C, OC, k, s, p, g):
    x = torch.randn(N, H, W, C, device=dev).to(BF)
    w = (torch.randn(OC, k, k, C // g, device=dev) * 0.05).to(BF)
    b = torch.randn(OC, device=dev)
    OH, OW = ops.conv_out_size(H, W, k, k, (s, s), (p, p, p, p))
    dy = torch.randn(N, OH, OW, OC, device=dev).to(BF)
    dw = torch.zeros(OC, k, k, C // g, device=dev)
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    t_f = timeit(lambda: ops.conv_fwd(x, w, b, (s, s), (p, p, p, p), g, 3))
    t_d = timeit(lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (s, s),
                                        (p, p, p, p), g)) if C >= 8 else 0
    t_w = timeit(lambda: ops.conv_wgrad(x, dy, dw, (s, s), (p, p, p, p), g))
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wn = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    t_tf = timeit(lambda: F.conv2d(xn, wn, None, s, p, 1, g))
    xr = xn.detach().requires_grad_(True)
    wr = wn.detach().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, p, 1, g)
    dyn = dy.permute(0, 3, 1, 2)
    t_tb = timeit(lambda: torch.autograd.grad(yr, (xr, wr), dyn,
                                              retain_graph=True))
    r = {"fwd_TF": fl / t_f / 1e12, "dgrad_TF": fl / t_d / 1e12 if t_d else 0,
         "wgrad_TF": fl / t_w / 1e12, "torch_fwd_TF": fl / t_tf / 1e12,
         "torch_bwd_TF": 2 * fl / t_tb / 1e12,
         "hvk_total_ms": (t_f + t_d + t_w) * 1e3,
         "torch_total_ms": (t_tf + t_tb) * 1e3}
    res[name] = r
    print(name, r, flush=True)


gemm_case("gemm_4096", 4096, 4096, 4096)
gemm_case("gemm_8192", 8192, 8192, 8192)
gemm_case("gemm_8192_nn", 8192, 8192, 8192, tb=False)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
gemm_case("fc6_fwd", B, 4096, 9216)
gemm_case("fc6_dgrad", B, 9216, 4096, tb=False)
gemm_case("fc6_wgrad", 4096, 9216, B, ta=True, tb=False)
conv_case("conv1", B, 227, 227, 3, 96, 11, 4, 0, 1)
conv_case("conv2", B, 27, 27, 96, 256, 5, 1, 2, 2)
conv_case("conv3", B, 13, 13, 256, 384, 3, 1, 1, 1)
conv_case("conv4", B, 13, 13, 384, 384, 3, 1, 1, 2)
conv_case("conv5", B, 13, 13, 384, 256, 3, 1, 1, 2)
conv_case("vgg_conv3_2", 64, 56, 56, 256, 256, 3, 1, 1, 1)
json.dump(res, open("gpurun_out/bench_kernels%s.json" % TAG, "w"),
          indent=1)
