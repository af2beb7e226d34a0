"""Same-process A/B of the fully-connected weight gradient at the bench
batch: dW = dY^T X (+ the bias gradient) as

* ``tn``: the library GEMM with both operands MN-major and the bias
  gradient from a ones column (the default, gd.py);
* ``nn``: dY transposed into a K-major copy first (a torch copy, timed),
  then the NN GEMM (K-major A: the 256 x 256 loop's fast loader) and the
  bias gradient by ops.col_sum;
* ``torch``: torch.mm on hipBLASLt (bf16 out, no bias gradient) as the
  vendor bar.

    python tools/bench_fc_wgrad_t.py [batch] [rounds]"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402

BF = torch.bfloat16


def timeit(fn, n=10, w=3):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    for name, n_in, n_out in (("fc6", 9216, 4096), ("fc7", 4096, 4096),
                              ("fc8", 4096, 1000)):
        e2 = (torch.randn(B, n_out, device="cuda") * 0.01).to(BF)
        x = torch.rand(B, n_in, device="cuda").to(BF)
        dw = torch.empty(n_out, n_in, device="cuda")
        db = torch.empty(n_out, device="cuda")
        e2t = torch.empty(n_out, B, device="cuda", dtype=BF)

        def tn():
            ops.gemm(e2, x, trans_a=True, out=dw, accumulate="overwrite",
                     bias_grad=db)

        def nn():
            e2t.copy_(e2.t())
            ops.gemm(e2t, x, out=dw, accumulate="overwrite")
            ops.col_sum(e2, out=db)

        def vendor():
            torch.mm(e2.t(), x)
        res = {"tn": [], "nn": [], "torch": []}
        for _ in range(rounds):
            for k, fn in (("tn", tn), ("nn", nn), ("torch", vendor)):
                res[k].append(timeit(fn))
        fl = 2.0 * B * n_in * n_out
        med = {k: statistics.median(v) for k, v in res.items()}
        print("%s b%d  " % (name, B) + "  ".join(
            "%s %.3f ms (%.0f TF)" % (k, v, fl / v / 1e9)
            for k, v in med.items()), flush=True)
        # the two library forms agree
        tn()
        ref_w, ref_b = dw.clone(), db.clone()
        nn()
        torch.cuda.synchronize()
        rel = float((dw - ref_w).norm() / (ref_w.norm() + 1e-12))
        relb = float((db - ref_b).norm() / (ref_b.norm() + 1e-12))
        print("   nn vs tn: rel %.2e (bias %.2e)" % (rel, relb), flush=True)


if __name__ == "__main__":
    main()
