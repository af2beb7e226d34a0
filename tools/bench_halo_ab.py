"""A/B of the LDS-halo stride-1 conv kernels (conv_halo.hip) against the
implicit GEMM on the AlexNet b1024 stride-1 shapes (conv1 after
space-to-depth, conv2..5) forward and backward-data, interleaved rounds in
one process, median TF (cdna_hip_programming.md §5.4 rule 24).

    python tools/bench_halo_ab.py [batch] [rounds]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))

import torch  # noqa: E402

from veles_amd import ops  # noqa: E402


def timeit(fn, n=10, w=2):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n * 1e-3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev, bf = "cuda", torch.bfloat16
    layers = {"conv1s2d": (B, 57, 57, 48, 96, 3, 0, 1),
              "conv2": (B, 27, 27, 96, 256, 5, 2, 2),
              "conv3": (B, 13, 13, 256, 384, 3, 1, 1),
              "conv4": (B, 13, 13, 384, 384, 3, 1, 2),
              "conv5": (B, 13, 13, 384, 256, 3, 1, 2)}
    out = {}
    for name, (N, H, W, C, OC, k, p, g) in layers.items():
        x = (torch.rand(N, H, W, C, device=dev) * 2 - 1).to(bf)
        w = ((torch.rand(OC, k, k, C // g, device=dev) * 2 - 1) * 0.05).to(bf)
        b = torch.randn(OC, device=dev)
        OH, OW = ops.conv_out_size(H, W, k, k, (1, 1), (p, p, p, p))
        dy = (torch.rand(N, OH, OW, OC, device=dev) * 2 - 1).to(bf)
        fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
        cases = {
            "fwd": lambda: ops.conv_fwd(x, w, b, (1, 1), (p, p, p, p), g, 3),
            "dgrad": lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1),
                                            (p, p, p, p), g, aux=x,
                                            aux_act=3)}
        for kind, fn in cases.items():
            ts = {0: [], 1: []}
            for _ in range(rounds):
                for h in (0, 1):
                    ops.set_conv_halo(bool(h), dgrad=bool(h))
                    ts[h].append(timeit(fn))
            ops.set_conv_halo(True, dgrad=False)
            med = {h: statistics.median(v) for h, v in ts.items()}
            key = "%s_%s" % (name, kind)
            out[key] = {"gemm_us": round(med[0] * 1e6, 1),
                        "halo_us": round(med[1] * 1e6, 1),
                        "gemm_tf": round(fl / med[0] / 1e12, 1),
                        "halo_tf": round(fl / med[1] / 1e12, 1)}
            print(key, out[key], flush=True)
        del x, w, dy
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
