"""FC weight gradient at AlexNet b1024: the bias gradient fused as a ones column
vs none vs a separate col_sum (median of 5 rounds).  python tools/bench_fc_wgrad_bias.py"""
import os, sys, statistics
sys.path.insert(0, os.getcwd())
import torch
from veles_amd import ops
def timeit(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / reps * 1e3
bf = torch.bfloat16
for name, K_in, N_out in (("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)):
    B = 1024
    x = (torch.rand(B, K_in, device="cuda") - 0.5).to(bf)
    dy = (torch.rand(B, N_out, device="cuda") - 0.5).to(bf)
    dw = torch.zeros(N_out, K_in, device="cuda")
    db = torch.zeros(N_out, device="cuda")
    f1 = lambda: ops.gemm(dy, x, trans_a=True, out=dw, accumulate="overwrite", bias_grad=db)
    f2 = lambda: ops.gemm(dy, x, trans_a=True, out=dw, accumulate="overwrite")
    f3 = lambda: (ops.gemm(dy, x, trans_a=True, out=dw, accumulate="overwrite"), ops.col_sum(dy, out=db))
    r = {1: [], 2: [], 3: []}
    for _ in range(5):
        r[1].append(timeit(f1)); r[2].append(timeit(f2)); r[3].append(timeit(f3))
    print(name, "fused-bias %.1f us, no-bias %.1f us, no-bias+col_sum %.1f us" % tuple(statistics.median(r[k]) for k in (1, 2, 3)), flush=True)
