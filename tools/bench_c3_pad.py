"""A/B for small-channel convolutions (VGG-16 conv1_1: C = 3): the packed
(kw, c)-run kernels against zero-padding the channels to 8 and running the
regular implicit-GEMM path.  Prints median ms per op and the max deviation
between the two results.

    python tools/bench_c3_pad.py [N] [H] [OC]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles_amd import ops  # noqa: E402


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 224
    OC = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    dev = "cuda"
    x = torch.randn(N, H, H, 3, device=dev).bfloat16()
    w = (torch.randn(OC, 3, 3, 3, device=dev) * 0.2).bfloat16()
    b = torch.randn(OC, device=dev)
    pad = (1, 1, 1, 1)
    y = torch.empty(N, H, H, OC, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(N, H, H, OC, device=dev).bfloat16()
    xp = F.pad(x, (0, 5)).contiguous()
    wp = F.pad(w, (0, 5)).contiguous()
    dw = torch.zeros(OC, 3, 3, 3, device=dev)
    dwp = torch.zeros(OC, 3, 3, 8, device=dev)
    db = torch.zeros(OC, device=dev)

    r = {}
    r["fwd_run"] = t(lambda: ops.conv_fwd(x, w, b, padding=pad, act="relu",
                                          out=y))
    y0 = y.clone()
    r["pad_x"] = t(lambda: F.pad(x, (0, 5)))
    r["fwd_pad8"] = t(lambda: ops.conv_fwd(xp, wp, b, padding=pad,
                                           act="relu", out=y))
    r["fwd_dev"] = (y.float() - y0.float()).abs().max().item()
    r["wgrad_run"] = t(lambda: (dw.zero_(), ops.conv_wgrad(
        x, dy, dw, padding=pad, dbias=db)))
    dw0 = dw.clone()
    r["wgrad_pad8"] = t(lambda: (dwp.zero_(), ops.conv_wgrad(
        xp, dy, dwp, padding=pad, dbias=db)))
    r["wgrad_dev"] = (dwp[..., :3] - dw0).abs().max().item() / \
        dw0.abs().max().item()
    for k, v in r.items():
        print("%-12s %.4f" % (k, v))


if __name__ == "__main__":
    main()
