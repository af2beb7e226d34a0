"""Probe: vendor-library bar on MI355X (torch eager, MIOpen convs, hipBLASLt GEMM).

Used only to know what the hand-written kernels must beat; not part of the framework.
"""
import json, time, torch, torch.nn as nn, torch.nn.functional as F
dev = "cuda"
print("device", torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).total_memory / 2**30, "GiB", flush=True)
res = {}
def t(fn, n=20, w=5):
    for _ in range(w): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n
for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (512, 4096, 9216), (9216, 4096, 512)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16); b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    dt = t(lambda: a @ b)
    res[f"mm_bf16_{M}x{N}x{K}_TF"] = 2 * M * N * K / dt / 1e12
    print(M, N, K, res[f"mm_bf16_{M}x{N}x{K}_TF"], flush=True)

class AlexNet(nn.Module):
    def __init__(s):
        super().__init__()
        s.c1 = nn.Conv2d(3, 96, 11, 4); s.c2 = nn.Conv2d(96, 256, 5, 1, 2, groups=2)
        s.c3 = nn.Conv2d(256, 384, 3, 1, 1); s.c4 = nn.Conv2d(384, 384, 3, 1, 1, groups=2)
        s.c5 = nn.Conv2d(384, 256, 3, 1, 1, groups=2)
        s.f6 = nn.Linear(9216, 4096); s.f7 = nn.Linear(4096, 4096); s.f8 = nn.Linear(4096, 1000)
    def forward(s, x):
        x = F.max_pool2d(F.local_response_norm(F.relu(s.c1(x)), 5, 1e-4, 0.75, 2), 3, 2)
        x = F.max_pool2d(F.local_response_norm(F.relu(s.c2(x)), 5, 1e-4, 0.75, 2), 3, 2)
        x = F.relu(s.c3(x)); x = F.relu(s.c4(x)); x = F.max_pool2d(F.relu(s.c5(x)), 3, 2)
        x = x.flatten(1)
        x = F.dropout(F.relu(s.f6(x)), 0.5); x = F.dropout(F.relu(s.f7(x)), 0.5)
        return s.f8(x)
for cl in (False, True):
    for B in (256, 512):
        m = AlexNet().to(dev)
        if cl: m = m.to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
        x = torch.randn(B, 3, 227, 227, device=dev)
        if cl: x = x.to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev)
        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
            opt.zero_grad(set_to_none=True); loss.backward(); opt.step()
        try:
            dt = t(step, n=10, w=3)
            res[f"alexnet_torch_amp_bf16_cl{int(cl)}_B{B}_img_s"] = B / dt
            print("alexnet cl", cl, "B", B, B / dt, "img/s", dt * 1e3, "ms", flush=True)
        except Exception as e:
            print("fail", cl, B, e, flush=True)
json.dump(res, open("gpurun_out/probe_torch_bar.json", "w"), indent=1)
