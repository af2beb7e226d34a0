"""A/B of the AlexNet b1024 fully-connected GEMMs: the library MFMA GEMM
(ops.gemm, with its fused bias / activation / activation-derivative /
overwrite-accumulate epilogues) against torch.matmul on the vendor library
(hipBLASLt) with the same fusions torch offers, interleaved rounds in one
process, median of the rounds (cdna_hip_programming.md rule 24).

    python tools/bench_fc_ab.py [batch] [rounds]
"""
import json
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
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = "cuda"
    bf = torch.bfloat16
    layers = [("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)]
    cases = {}
    for name, K, N in layers:
        x = torch.randn(B, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.01).to(bf)
        bias = torch.randn(N, device=dev)
        y = torch.empty(B, N, device=dev, dtype=bf)
        e = torch.randn(B, N, device=dev).to(bf)
        yref = torch.relu(torch.randn(B, N, device=dev)).to(bf)
        dx = torch.empty(B, K, device=dev, dtype=bf)
        gw = torch.empty(N, K, device=dev, dtype=torch.float32)
        gb = torch.empty(N, device=dev, dtype=torch.float32)
        bias_bf = bias.to(bf)
        flops = 2.0 * B * N * K
        ours = {
            "fwd": lambda x=x, w=w, bias=bias, y=y: ops.gemm(
                x, w, trans_b=True, out=y, bias=bias, act=3),
            "dgrad": lambda e=e, w=w, dx=dx, yref=yref, x=x: ops.gemm(
                e, w, out=dx, aux=x, aux_act=3),
            "wgrad": lambda e=e, x=x, gw=gw, gb=gb: ops.gemm(
                e, x, trans_a=True, out=gw, accumulate="overwrite",
                bias_grad=gb),
        }
        try:
            torch.mm(e.t(), x, out_dtype=torch.float32)
            f32out = True
        except Exception:  # noqa: BLE001
            f32out = False
        vend = {
            "fwd": lambda x=x, w=w, b=bias_bf: torch._addmm_activation(
                b, x, w.t()),
            "dgrad": lambda e=e, w=w, x=x: (e @ w) * (x > 0),
            "wgrad": (lambda e=e, x=x: (torch.mm(e.t(), x,
                                                 out_dtype=torch.float32),
                                        e.float().sum(0)))
            if f32out else (lambda e=e, x=x: (e.t() @ x, e.float().sum(0))),
        }
        for k in ours:
            cases["%s_%s" % (name, k)] = (ours[k], vend[k], flops)
    res = {k: ([], []) for k in cases}
    for _ in range(rounds):
        for k, (fo, fv, _) in cases.items():
            res[k][0].append(timeit(fo))
            res[k][1].append(timeit(fv))
    out = {"batch": B, "rounds": rounds, "wgrad_vendor_f32_out": f32out,
           "cases": {}}
    for k, (a, b) in res.items():
        fl = cases[k][2]
        ma, mb = statistics.median(a), statistics.median(b)
        out["cases"][k] = {"ours_us": round(ma, 1), "vendor_us": round(mb, 1),
                           "ours_tf": round(fl / ma / 1e6, 1),
                           "vendor_tf": round(fl / mb / 1e6, 1)}
        print("%-12s ours %7.1f us (%6.1f TF)   vendor %7.1f us (%6.1f TF)" %
              (k, ma, fl / ma / 1e6, mb, fl / mb / 1e6), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
