"""A few launches of the weight-stationary convs (AlexNet conv2 / conv1
forward, VGG conv1_2 backward-data) for rocprofv3 --pmc passes."""
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

BF = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(BF)


x = r(B, 27, 27, 96)
w = (r(256, 5, 5, 48) * 0.05).to(BF)
y = torch.empty(B, 27, 27, 256, device="cuda", dtype=BF)
b = torch.randn(256, device="cuda")
x1 = r(B, 227, 227, 3)
w1 = (r(96, 11, 11, 3) * 0.05).to(BF)
y1 = torch.empty(B, 55, 55, 96, device="cuda", dtype=BF)
dy = r(B // 8, 224, 224, 64)
wv = (r(64, 3, 3, 64) * 0.05).to(BF)
dx = torch.empty(B // 8, 224, 224, 64, device="cuda", dtype=BF)
for _ in range(3):
    ops.conv_fwd(x, w, b, (1, 1), (2, 2, 2, 2), 2, "str", out=y)
    ops.conv_fwd(x1, w1, b[:96], (4, 4), (0, 0, 0, 0), 1, "str", out=y1)
    ops.conv_dgrad(dy, wv, (B // 8, 224, 224, 64), (1, 1), (1, 1, 1, 1), 1,
                   aux=dy, aux_act="str", out=dx)
torch.cuda.synchronize()
print("ok")
