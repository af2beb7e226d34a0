"""Weight-stationary convolution kernels (csrc/kernels/conv_ws.hip) against
the float32 PyTorch references (F.conv2d / torch.nn.grad.conv2d_input on
the same bf16 values) and against the implicit-GEMM path they replace
(ops.set_conv_ws(False)): AlexNet conv2 forward (5 x 5, groups 2, full-row
windows with tiles across images), conv1 forward through the space-to-depth
image, VGG conv1_2 forward and backward-data (224-wide segment windows)
with the ReLU derivative of the layer below."""
import pytest
import torch
import torch.nn.functional as F

from veles_amd import ops

pytestmark = pytest.mark.gpu


def _r(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return ((torch.rand(*shape, generator=g, device="cuda") - 0.5) *
            scale).to(torch.bfloat16)


def _fwd_ref(x, w, b, stride, pad, groups, relu):
    y = F.conv2d(F.pad(x.permute(0, 3, 1, 2).float(), (pad,) * 4),
                 w.permute(0, 3, 1, 2).float(), b, stride=stride,
                 groups=groups)
    if relu:
        y = y.clamp_min(0)
    return y.permute(0, 2, 3, 1)


def _both(fn):
    out = {}
    try:
        for on in (True, False):
            ops.set_conv_ws(on)
            out[on] = fn()
            torch.cuda.synchronize()
    finally:
        ops.set_conv_ws(False)
    return out


def _close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    assert err <= tol * (b.abs().max().item() + 1e-6), err


@pytest.mark.parametrize("shape", [
    # N, H, W, C, OC, K, stride, pad, groups
    (3, 27, 27, 96, 256, 5, 1, 2, 2),      # AlexNet conv2
    (2, 227, 227, 3, 96, 11, 4, 0, 1),     # AlexNet conv1 (space-to-depth)
    (1, 224, 224, 64, 64, 3, 1, 1, 1),     # VGG conv1_2
])
def test_conv_ws_forward(shape):
    N, H, W, C, OC, K, st, pad, g = shape
    x = _r(N, H, W, C, scale=2.0, seed=1)
    w = _r(OC, K, K, C // g, scale=0.2, seed=2)
    b = torch.randn(OC, device="cuda") * 0.1
    res = _both(lambda: ops.conv_fwd(x, w, b, (st, st), (pad,) * 4, g,
                                     act="str"))
    ref = _fwd_ref(x, w, b, st, pad, g, True)
    _close(res[True], ref, 1e-2)
    # the same MFMA K order as the implicit GEMM: equal to bf16 rounding
    _close(res[True], res[False], 1e-2)
    assert (res[True].float() - res[False].float()).abs().max().item() <= \
        4e-3 * res[False].float().abs().max().item()


def test_conv_ws_dgrad_vgg_conv1_2():
    N, H, W, C, OC = 1, 224, 224, 64, 64
    dy = _r(N, H, W, OC, scale=1.0, seed=3)
    w = _r(OC, 3, 3, C, scale=0.2, seed=4)
    aux = _r(N, H, W, C, scale=2.0, seed=5)   # the layer below's ReLU output
    res = _both(lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1),
                                       (1, 1, 1, 1), 1, aux=aux,
                                       aux_act="str"))
    ref = torch.nn.grad.conv2d_input(
        (N, C, H, W), w.permute(0, 3, 1, 2).float(),
        dy.permute(0, 3, 1, 2).float(), padding=1).permute(0, 2, 3, 1)
    ref = ref * (aux.float() > 0)
    _close(res[True], ref, 1e-2)
    _close(res[True], res[False], 4e-3)


def test_conv_ws_taken():
    from veles_amd.ops import _lib
    x = _r(2, 27, 27, 96, scale=1.0, seed=1)
    w = _r(256, 5, 5, 48, scale=0.1, seed=2)
    y = torch.empty(2, 27, 27, 256, dtype=torch.bfloat16, device="cuda")
    rc = _lib.lib().hvk_conv_fwd_ws(
        x.data_ptr(), w.data_ptr(), None, y.data_ptr(), 2, 27, 27, 96, 256,
        5, 5, 2, 2, 27, 27, 2, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    # a shape without a weight-stationary variant is left to the caller
    rc = _lib.lib().hvk_conv_fwd_ws(
        x.data_ptr(), w.data_ptr(), None, y.data_ptr(), 2, 27, 27, 96, 256,
        3, 3, 1, 1, 27, 27, 2, 0, torch.cuda.current_stream().cuda_stream)
    assert rc == -2
