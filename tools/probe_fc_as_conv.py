import statistics, sys
import torch
sys.path.insert(0, ".")
import veles_amd.ops as ops
from veles_amd.ops import _lib
BF = torch.bfloat16
def timeit(fn, n=20, w=3):
    for _ in range(w): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3
lib = _lib.lib()
B = 3072
for name, K, N in (("fc6", 9216, 4096), ("fc7", 4096, 4096)):
    x = torch.randn(B, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.01).to(BF)
    bias = torch.randn(N, device="cuda")
    y = torch.empty(B, N, device="cuda", dtype=BF)
    y2 = torch.empty(1, 1, B, N, device="cuda", dtype=BF)
    x4, w4 = x.view(1, 1, B, K), w.view(N, 1, 1, K)
    gem = lambda: ops.gemm(x, w, trans_b=True, out=y, bias=bias, act=3)
    res = {"gemm": [], "conv_default": [], "conv_t4_1": [], "conv_t4_2": []}
    for _ in range(5):
        lib.hvk_set_gemm_variant(-1); res["gemm"].append(timeit(gem))
        lib.hvk_set_gemm_variant(-1); res["conv_default"].append(timeit(lambda: ops.conv_fwd(x4, w4, bias, (1, 1), (0, 0, 0, 0), 1, "str", out=y2)))
        lib.hvk_set_gemm_variant(51); res["conv_t4_1"].append(timeit(lambda: ops.conv_fwd(x4, w4, bias, (1, 1), (0, 0, 0, 0), 1, "str", out=y2)))
        lib.hvk_set_gemm_variant(52); res["conv_t4_2"].append(timeit(lambda: ops.conv_fwd(x4, w4, bias, (1, 1), (0, 0, 0, 0), 1, "str", out=y2)))
    lib.hvk_set_gemm_variant(-1)
    fl = 2.0 * B * N * K
    gem(); ref = y.clone()
    for v in (51,):
        lib.hvk_set_gemm_variant(v); ops.conv_fwd(x4, w4, bias, (1, 1), (0, 0, 0, 0), 1, "str", out=y2)
    lib.hvk_set_gemm_variant(-1); torch.cuda.synchronize()
    rel = float((y2.view(B, N).float() - ref.float()).norm() / ref.float().norm())
    print(name, "  ".join("%s %.1f us (%.0f TF)" % (k, statistics.median(v), fl / statistics.median(v) / 1e6) for k, v in res.items()), "rel(t4 vs gemm) %.1e" % rel, flush=True)
