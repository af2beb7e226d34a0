"""hvk_softmax_ce at AlexNet's shape (b3072 x 1000 classes, bf16 logits and
error): the register-cached row (default) against the three-pass loop
(hvk_gemm_variant 65), HIP-event time and bit-identity of every output.

    python tools/probe_softmax_ce.py [batch] [classes]"""
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn(B, C, generator=g, device="cuda") * 4).to(torch.bfloat16)
    x[5, 7] = x[5, 9] = 30.0   # an argmax tie
    lab = torch.randint(0, C, (B,), generator=g, device="cuda",
                        dtype=torch.int32)
    lib = ops._lib.lib()
    res = {}
    for v in (65, -1):
        lib.hvk_set_gemm_variant(v)
        err = torch.empty(B, C, dtype=torch.bfloat16, device="cuda")
        probs = torch.empty(B, C, device="cuda")
        mi = torch.empty(B, dtype=torch.int32, device="cuda")
        met = torch.zeros(3, device="cuda")

        def f():
            ops.softmax_ce(x, lab, err=err, probs=probs, max_idx=mi,
                           metrics=met)
        for _ in range(20):
            f()
        met.zero_()
        f()
        torch.cuda.synchronize()
        res[v] = (err.clone(), probs.clone(), mi.clone(), met.clone())
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        for _ in range(50):
            f()
        b.record()
        b.synchronize()
        print("softmax_ce b%d C%d variant %d: %.1f us" % (
            B, C, v, a.elapsed_time(b) / 50 * 1e3))
    lib.hvk_set_gemm_variant(-1)
    same = all(torch.equal(p, q) for p, q in zip(res[65][:3], res[-1][:3]))
    print("err / probs / argmax bit-identical: %s; metrics %s vs %s" % (
        same, res[65][3].tolist(), res[-1][3].tolist()))


if __name__ == "__main__":
    main()
