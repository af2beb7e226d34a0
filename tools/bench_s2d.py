"""Time the space-to-depth of AlexNet's conv1 input at batch 1024 (median
of 20 HIP-event timings).  HVK_S2D_CHUNK=0 selects the pixel-per-lane
kernel instead of the chunk-per-lane one (profiles/s2d_chunk_r2/).

    python tools/bench_s2d.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles_amd import ops  # noqa: E402


def main():
    x = torch.randn(1024, 227, 227, 3, device="cuda").bfloat16()

    def f():
        return ops.space_to_depth(x, 4, 11, 11, (0, 0, 0, 0))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        f()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print("s2d b1024 ms", ts[10])


if __name__ == "__main__":
    main()
