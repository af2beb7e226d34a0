"""Halo weight-gradient kernel (csrc/kernels/wgrad_halo.hip) against the
float32 PyTorch reference (torch.nn.grad.conv2d_weight on the same bf16
values): AlexNet conv2-5 geometries at small batches, pixel splits that
cut images at arbitrary rows (a step then spans two images), accumulation
into a non-zero dW, the fused bias gradient, and bit-stability run to run
(workspace slices summed in split order, no atomics)."""
import pytest
import torch
import torch.nn.functional as F

from veles_amd import ops
from veles_amd.ops import _lib

pytestmark = pytest.mark.gpu

# (N, H, W, C, OC, K, pad, groups)
SHAPES = {
    "conv3": (4, 13, 13, 256, 384, 3, 1, 1),
    "conv4": (3, 13, 13, 384, 384, 3, 1, 2),
    "conv5": (5, 13, 13, 384, 256, 3, 1, 2),
    "conv2": (2, 27, 27, 96, 256, 5, 2, 2),
    "wide": (2, 20, 20, 128, 128, 3, 1, 1),
    "vgg28": (2, 28, 28, 256, 256, 3, 1, 1),
    "vgg56": (2, 56, 56, 128, 256, 3, 1, 1),
    # segment windows: 112 / 224-wide VGG layers, AlexNet conv1's s2d image
    "vgg112": (1, 112, 112, 64, 128, 3, 1, 1),
    "vgg224": (1, 224, 224, 64, 64, 3, 1, 1),
    "s2d55": (3, 57, 57, 48, 96, 3, 0, 1),
}


def _ref(x, dy, K, pad, groups):
    N, H, W, C = x.shape
    OC = dy.shape[3]
    xp = F.pad(x.permute(0, 3, 1, 2).float(), (pad, pad, pad, pad))
    g = torch.nn.grad.conv2d_weight(xp, (OC, C // groups, K, K),
                                    dy.permute(0, 3, 1, 2).float(),
                                    groups=groups)
    return g.permute(0, 2, 3, 1).contiguous(), dy.float().reshape(-1, OC).sum(0)


def _data(shape, seed):
    N, H, W, C, OC, K, pad, groups = shape
    OH, OW = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.rand(N, H, W, C, generator=g, device="cuda") - 0.5).to(
        torch.bfloat16)
    dy = (torch.rand(N, OH, OW, OC, generator=g, device="cuda") - 0.5).to(
        torch.bfloat16)
    return x, dy


def _halo(x, dy, dw, db, K, pad, groups, splits=0):
    N, H, W, C = x.shape
    _, OH, OW, OC = dy.shape
    fn = _lib.lib().hvk_conv_wgrad_halo
    geo = (N, H, W, C, OC, K, K, pad, pad, OH, OW, groups, splits)
    need = fn(x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
              0 if db is None else db.data_ptr(), None, *geo,
              torch.cuda.current_stream().cuda_stream)
    assert need > 0, "shape does not take the halo kernel"
    ws = torch.empty(int(need), dtype=torch.float32, device="cuda")
    rc = fn(x.data_ptr(), dy.data_ptr(), dw.data_ptr(),
            0 if db is None else db.data_ptr(), ws.data_ptr(), *geo,
            torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    return _lib.lib().hvk_conv_wgrad_halo_splits(*geo)


@pytest.mark.parametrize("name", sorted(SHAPES))
@pytest.mark.parametrize("splits", [0, 7])
def test_halo_wgrad_matches_fp32(name, splits):
    shape = SHAPES[name]
    N, H, W, C, OC, K, pad, groups = shape
    x, dy = _data(shape, 11)
    ref_w, ref_b = _ref(x, dy, K, pad, groups)
    dw0 = torch.randn(OC, K, K, C // groups, device="cuda")
    db0 = torch.randn(OC, device="cuda")
    dw, db = dw0.clone(), db0.clone()
    sp = _halo(x, dy, dw, db, K, pad, groups, splits)
    torch.cuda.synchronize()
    assert sp >= 1
    scale = ref_w.abs().max().item()
    err = (dw - dw0 - ref_w).abs().max().item()
    assert err <= 2e-5 * max(scale, 1.0) * (dy.numel() / OC) ** 0.5, \
        (err, scale)
    berr = (db - db0 - ref_b).abs().max().item()
    assert berr <= 1e-3 * max(ref_b.abs().max().item(), 1.0), berr


def test_halo_wgrad_bit_stable_and_no_bias():
    shape = SHAPES["conv3"]
    N, H, W, C, OC, K, pad, groups = shape
    x, dy = _data(shape, 5)
    outs = []
    for _ in range(2):
        dw = torch.zeros(OC, K, K, C, device="cuda")
        _halo(x, dy, dw, None, K, pad, groups)
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref_w, _ = _ref(x, dy, K, pad, groups)
    assert torch.allclose(outs[0], ref_w, rtol=1e-3, atol=1e-2)


def test_conv_wgrad_takes_halo_and_matches_old_path():
    """ops.conv_wgrad routes stride-1 bf16 shapes to the halo kernel; the
    result equals the 128-row / T4 loop's to f32 rounding."""
    shape = SHAPES["conv5"]
    N, H, W, C, OC, K, pad, groups = shape
    x, dy = _data(shape, 3)
    res = {}
    try:
        for on in (True, False):
            ops.set_halo_wgrad(on)
            dw = torch.zeros(OC, K, K, C // groups, device="cuda")
            db = torch.zeros(OC, device="cuda")
            ops.conv_wgrad(x, dy, dw, padding=(pad,) * 4, groups=groups,
                           dbias=db)
            res[on] = (dw, db)
    finally:
        ops.set_halo_wgrad(True)
    torch.cuda.synchronize()
    assert torch.allclose(res[True][0], res[False][0], rtol=1e-4, atol=1e-3)
    assert torch.allclose(res[True][1], res[False][1], rtol=1e-4, atol=1e-3)
