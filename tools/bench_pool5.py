"""Same-process A/B of the 3x3 / stride-2 max-pool backward (AlexNet pool5,
13x13x256 -> 6x6 at batch B): the 2x2-block kernel (variant 0) against the
per-pixel kernel (variant 1), HIP-event median of 5 interleaved rounds.

    python tools/bench_pool5.py [batch]"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = ops._lib.lib()
    shape = (B, 13, 13, 256)
    x = torch.relu(torch.randn(*shape, device="cuda")).to(torch.bfloat16)
    y, am = ops.pool_fwd(x, 3, 3, (2, 2), "max")
    dy = torch.randn(*y.shape, device="cuda").to(torch.bfloat16)
    dx = torch.empty_like(x)
    f = lambda: ops.pool_bwd(dy, am, shape, 3, 3, (2, 2), "max", aux=x,  # noqa
                             aux_act=3, out=dx)
    ts = {0: [], 1: []}
    try:
        for _ in range(5):
            for v in (0, 1):
                lib.hvk_set_pool_bwd_variant(v)
                ts[v].append(timeit(f))
    finally:
        lib.hvk_set_pool_bwd_variant(0)
    mb = (x.numel() * 2 * 2 + dy.numel() * 2 + am.numel() * 4) / 1e6
    for v, name in ((0, "2x2 blocks"), (1, "per pixel")):
        us = statistics.median(ts[v])
        print("pool5 bwd %-10s %.1f us  (%.0f MB min traffic, %.2f TB/s)" % (
            name, us, mb, mb / us))


if __name__ == "__main__":
    main()
