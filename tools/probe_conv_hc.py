"""A few launches of the channel-chunked halo convs and the kernels they
compete with (AlexNet conv3 forward on conv_hc configuration 6 and on the
implicit GEMM, conv2 forward / backward-data on conv_hc) for rocprofv3
--pmc passes (tools/gpu_pmc_hc.sh)."""
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402

BF = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(BF)


x3 = r(B, 13, 13, 256)
w3 = (r(384, 3, 3, 256) * 0.05).to(BF)
b3 = torch.randn(384, device="cuda")
y3 = torch.empty(B, 13, 13, 384, device="cuda", dtype=BF)
x2 = r(B, 27, 27, 96)
w2 = (r(256, 5, 5, 48) * 0.05).to(BF)
b2 = torch.randn(256, device="cuda")
y2 = torch.empty(B, 27, 27, 256, device="cuda", dtype=BF)
dy2 = r(B, 27, 27, 256)
dx2 = torch.empty(B, 27, 27, 96, device="cuda", dtype=BF)
for _ in range(3):
    ops.set_conv_hc(True, -1)
    ops.conv_fwd(x3, w3, b3, (1, 1), (1, 1, 1, 1), 1, "str", out=y3)
    ops.set_conv_hc(False, -2)
    ops.conv_fwd(x3, w3, b3, (1, 1), (1, 1, 1, 1), 1, "str", out=y3)
    ops.set_conv_hc(True, -2)
    ops.conv_fwd(x2, w2, b2, (1, 1), (2, 2, 2, 2), 2, "str", out=y2)
    ops.conv_dgrad(dy2, w2, (B, 27, 27, 96), (1, 1), (2, 2, 2, 2), 2,
                   aux=x2, aux_act="str", out=dx2)
torch.cuda.synchronize()
