"""hvk_dropout at AlexNet's fc6 / fc7 shape (b3072 x 4096 bf16): the 8-wide
path (default) against the per-element kernel (hvk_gemm_variant 66), HIP-event
time and bit-identity, host seed and device seed with a mask offset.

    python tools/probe_dropout.py [batch] [features]"""
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, F, generator=g, device="cuda").to(torch.bfloat16)
    sd = torch.tensor([12345], dtype=torch.int32, device="cuda")
    lib = ops._lib.lib()
    outs = {}
    for v in (66, -1):
        lib.hvk_set_gemm_variant(v)
        y = torch.empty_like(x)
        y2 = torch.empty_like(x)
        for f in (lambda: ops.dropout(x, 0.5, 777, out=y),
                  lambda: ops.dropout(x, 0.5, 0, out=y2, seed_dev=sd,
                                      base=4096)):
            for _ in range(20):
                f()
        torch.cuda.synchronize()
        outs[v] = (y.clone(), y2.clone())
        f = lambda: ops.dropout(x, 0.5, 777, out=y)  # noqa: E731
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        for _ in range(50):
            f()
        b.record()
        b.synchronize()
        print("dropout b%d x %d variant %d: %.1f us" % (
            B, F, v, a.elapsed_time(b) / 50 * 1e3))
    lib.hvk_set_gemm_variant(-1)
    print("bit-identical (host seed, device seed + base): %s, %s; kept "
          "fraction %.4f" % (torch.equal(outs[66][0], outs[-1][0]),
                             torch.equal(outs[66][1], outs[-1][1]),
                             (outs[-1][0] != 0).float().mean().item()))


if __name__ == "__main__":
    main()
