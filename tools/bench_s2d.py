import torch, sys
sys.path.insert(0, '.')
from veles_amd import ops
x = torch.randn(1024, 227, 227, 3, device='cuda').bfloat16()
f = lambda: ops.space_to_depth(x, 4, 11, 11, (0, 0, 0, 0))
for _ in range(3): f()
torch.cuda.synchronize()
ts = []
for _ in range(20):
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record(); f(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b))
ts.sort(); print("s2d b1024 ms", ts[10])
