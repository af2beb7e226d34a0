"""Split-K sweep for the FC forward GEMMs (bias + activation epilogue):
time ops.gemm at forced split counts (0 = the unsplit kernel), median of
interleaved rounds.  python tools/bench_splitk_sweep.py [batch] [rounds]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))

import torch  # noqa: E402

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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    bf = torch.bfloat16
    for name, K, N, act in (("fc6", 9216, 4096, 1), ("fc7", 4096, 4096, 1),
                            ("fc8", 4096, 1000, 0)):
        x = (torch.rand(B, K, device="cuda") - 0.5).to(bf)
        w = ((torch.rand(N, K, device="cuda") - 0.5) * 0.02).to(bf)
        bias = torch.randn(N, device="cuda")
        out = torch.empty(B, N, device="cuda", dtype=bf)
        res = {}
        for sk in (0, 2, 3, 4, 6, 8):
            res[sk] = []

        def run(sk):
            ops._splitk_forced = sk
            try:
                ops.gemm(x, w, trans_b=True, bias=bias, act=act, out=out)
            finally:
                ops._splitk_forced = None
        for _ in range(rounds):
            for sk in res:
                res[sk].append(timeit(lambda: run(sk)))
        fl = 2.0 * B * N * K
        print(name, " ".join("sk%d=%.1fus(%.0fTF)" % (
            sk, statistics.median(v), fl / statistics.median(v) / 1e6)
            for sk, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
