"""Time the memory-bound kernels of the AlexNet step on their real shapes
(and PyTorch equivalents where one exists) -> JSON lines."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    res = {}
    x = torch.randn(B, 55, 55, 96, device=DEV).to(BF)
    am = torch.empty(B, 27, 27, 96, dtype=torch.int32, device=DEV)
    y = torch.empty(B, 27, 27, 96, dtype=BF, device=DEV)
    gb = (x.numel() * 2 + y.numel() * 6) / 1e9
    res["pool1_fwd"] = bench(lambda: ops.pool_fwd(x, 3, 3, (2, 2), "max",
                                                  out=y, argmax=am))
    res["pool1_fwd_noargmax"] = bench(lambda: ops.pool_fwd(
        x, 3, 3, (2, 2), "max", out=y, argmax=None))
    xc = x.permute(0, 3, 1, 2)
    res["torch_maxpool1_channels_last"] = bench(
        lambda: torch.nn.functional.max_pool2d(xc, 3, 2))
    res["pool1_GB"] = gb
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    res["pool1_bwd"] = bench(lambda: ops.pool_bwd(
        dy, am, tuple(x.shape), 3, 3, (2, 2), "max", out=dx))
    res["lrn1_fwd"] = bench(lambda: ops.lrn_fwd(x, 5, 2e-5, 0.75, 1.0,
                                                out=dx))
    res["lrn1_bwd"] = bench(lambda: ops.lrn_bwd(x, x, 5, 2e-5, 0.75, 1.0,
                                                out=dx))
    img = torch.randn(B, 227, 227, 3, device=DEV).to(BF)
    res["s2d"] = bench(lambda: ops.space_to_depth(img, 4, 11, 11,
                                                  (0, 0, 0, 0)))
    src = torch.randint(0, 255, (B * 2, 227 * 227 * 3), dtype=torch.uint8,
                        device=DEV)
    sh = torch.randperm(B * 2, device=DEV).to(torch.int32)
    mean = torch.rand(227 * 227 * 3, device=DEV)
    dst = torch.empty(B, 227 * 227 * 3, dtype=BF, device=DEV)
    res["fill"] = bench(lambda: ops.fill_minibatch(src, sh, 0, B, dst,
                                                   mean=mean, rdisp=mean))
    big = torch.empty(1 << 28, dtype=torch.uint8, device=DEV)
    big2 = torch.empty_like(big)
    res["copy_256MB_us"] = bench(lambda: big2.copy_(big))
    for k, v in res.items():
        print(json.dumps({"kernel": k, "us": round(v, 1)}))


if __name__ == "__main__":
    main()
