"""FC weight gradient at AlexNet b3072: the TN GEMM with the fused bias
ones column (the default, dW = dY^T x) against dY transposed first and the
NN GEMM (pp256 loop), per layer; HIP-event times.

    python tools/probe_fc_wgrad_nn.py [batch]"""
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402


def timeit(f, reps=30):
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    for name, nin, nout in (("fc6", 9216, 4096), ("fc7", 4096, 4096),
                            ("fc8", 4096, 1000)):
        x = torch.randn(B, nin, device="cuda").to(torch.bfloat16)
        e = torch.randn(B, nout, device="cuda").to(torch.bfloat16)
        gw = torch.empty(nout, nin, device="cuda")
        gb = torch.empty(nout, device="cuda")
        et = e.t().contiguous()
        tn = timeit(lambda: ops.gemm(e, x, trans_a=True, out=gw,
                                     accumulate="overwrite", bias_grad=gb))
        ref, refb = gw.clone(), gb.clone()
        nn = timeit(lambda: ops.gemm(et, x, out=gw, accumulate="overwrite"))
        err = ((gw - ref).norm() / ref.norm()).item()
        fl = 2.0 * B * nin * nout
        line = "%s b%d: TN+bias %.1f us (%.0f TF), NN %.1f us (%.0f TF)" % (
            name, B, tn, fl / tn / 1e6, nn, fl / nn / 1e6)
        if nout % 64 == 0:
            ws = torch.empty(B // 64 * nout, device="cuda")
            tc = timeit(lambda: ops.transpose_colsum(e, out=et, colsum=gb,
                                                     ws=ws))
            same_t = torch.equal(et, e.t())
            berr = ((gb - refb).norm() / refb.norm()).item()
            line += (", transpose+colsum %.1f us (transpose exact %s, bias "
                     "rel diff %.1e)" % (tc, same_t, berr))
        print(line + ", weight rel diff %.1e" % err)


if __name__ == "__main__":
    main()
