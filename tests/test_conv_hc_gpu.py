"""Channel-chunked halo convolutions (csrc/kernels/conv_hc.hip) against the
float32 PyTorch references (F.conv2d / torch.nn.grad.conv2d_input on the
same bf16 values) and against the kernels they replace
(ops.set_conv_hc(False)): every AlexNet conv forward (conv1 through the
space-to-depth image) and the stride-1 backward-data shapes, partial last
tiles, tiles spanning several images, and batches large enough that every
persistent workgroup walks several items."""
import pytest
import torch
import torch.nn.functional as F

from veles_amd import ops

pytestmark = pytest.mark.gpu


def _r(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return ((torch.rand(*shape, generator=g, device="cuda") - 0.5) *
            scale).to(torch.bfloat16)


def _both(fn):
    out = {}
    prev = ops._CONV_HC
    try:
        for on in (True, False):
            ops.set_conv_hc(on, -1)   # every supported shape
            out[on] = fn()
            torch.cuda.synchronize()
    finally:
        ops.set_conv_hc(prev, -2)
    return out


def _close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    assert err <= tol * (b.abs().max().item() + 1e-6), err


FWD = [
    # N, H, W, C, OC, K, stride, pad, groups
    (2, 227, 227, 3, 96, 11, 4, 0, 1),     # conv1 (space-to-depth)
    (3, 27, 27, 96, 256, 5, 1, 2, 2),      # conv2
    (3, 13, 13, 256, 384, 3, 1, 1, 1),     # conv3
    (3, 13, 13, 384, 384, 3, 1, 1, 2),     # conv4
    (3, 13, 13, 384, 256, 3, 1, 1, 2),     # conv5
    (384, 13, 13, 384, 384, 3, 1, 1, 2),   # conv4, many items per workgroup
    (1, 56, 56, 64, 64, 3, 1, 1, 1),       # VGG-16 64-channel layer
    (1, 224, 224, 64, 64, 3, 1, 1, 1),     # VGG-16 conv1_2: 224-wide window
    (2, 28, 28, 256, 512, 3, 1, 1, 1),     # VGG-16 conv4_1
    (2, 14, 14, 512, 512, 3, 1, 1, 1),     # VGG-16 conv5_x
]


@pytest.mark.parametrize("shape", FWD)
def test_conv_hc_forward(shape):
    N, H, W, C, OC, K, st, pad, g = shape
    x = _r(N, H, W, C, scale=2.0, seed=1)
    w = _r(OC, K, K, C // g, scale=0.2, seed=2)
    b = torch.randn(OC, device="cuda") * 0.1
    res = _both(lambda: ops.conv_fwd(x, w, b, (st, st), (pad,) * 4, g,
                                     act="str"))
    ref = F.conv2d(F.pad(x.permute(0, 3, 1, 2).float(), (pad,) * 4),
                   w.permute(0, 3, 1, 2).float(), b, stride=st,
                   groups=g).clamp_min(0).permute(0, 2, 3, 1)
    _close(res[True], ref, 1e-2)
    _close(res[True], res[False], 1e-2)


DGRAD = [
    (3, 27, 27, 96, 256, 5, 2, 2),         # conv2
    (3, 13, 13, 256, 384, 3, 1, 1),        # conv3
    (3, 13, 13, 384, 384, 3, 1, 2),        # conv4
    (3, 13, 13, 384, 256, 3, 1, 2),        # conv5
    (200, 27, 27, 96, 256, 5, 2, 2),       # conv2, many items per workgroup
    (2, 56, 56, 128, 256, 3, 1, 1),        # VGG-16 conv3_1 backward-data
    (2, 28, 28, 256, 512, 3, 1, 1),        # VGG-16 conv4_1
    (2, 14, 14, 512, 512, 3, 1, 1),        # VGG-16 conv5_x
    (1, 224, 224, 64, 64, 3, 1, 1),        # VGG-16 conv1_2: 224-wide window
]


@pytest.mark.parametrize("shape", DGRAD)
def test_conv_hc_dgrad(shape):
    N, H, W, C, OC, K, pad, g = shape
    dy = _r(N, H, W, OC, scale=1.0, seed=3)
    w = _r(OC, K, K, C // g, scale=0.2, seed=4)
    aux = _r(N, H, W, C, scale=2.0, seed=5)   # the layer below's ReLU output
    res = _both(lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1),
                                       (pad,) * 4, g, aux=aux,
                                       aux_act="str"))
    ref = torch.nn.grad.conv2d_input(
        (N, C, H, W), w.permute(0, 3, 1, 2).float(),
        dy.permute(0, 3, 1, 2).float(), padding=pad,
        groups=g).permute(0, 2, 3, 1)
    ref = ref * (aux.float() > 0)
    _close(res[True], ref, 1e-2)
    _close(res[True], res[False], 1e-2)


def test_conv_hc_taken_and_forced_variants():
    from veles_amd.ops import _lib
    lib = _lib.lib()
    x = _r(3, 13, 13, 384, scale=1.0, seed=1)
    w = _r(384, 3, 3, 192, scale=0.1, seed=2)
    ref = None
    # the 16x16x32 configurations (conv_hc32 needs a packed-weight
    # workspace, which these direct calls do not pass)
    lib.hvk_hc32(0)
    try:
        # conv4 fits the 128-, 96- and 64-channel tiles: every forced
        # configuration gives the same sums up to rounding
        for var in (-1, 2, 3):
            lib.hvk_hc_variant(var)
            y = torch.empty(3, 13, 13, 384, dtype=torch.bfloat16,
                            device="cuda")
            rc = lib.hvk_conv_fwd_hc(
                x.data_ptr(), w.data_ptr(), None, y.data_ptr(), 3, 13, 13,
                384, 384, 3, 3, 1, 1, 13, 13, 2, 0, None,
                torch.cuda.current_stream().cuda_stream)
            assert rc == 0, var
            torch.cuda.synchronize()
            if ref is None:
                ref = y
            else:
                _close(y, ref, 4e-3)
        # AlexNet conv2 on the 5 x 5 tiles with and without the kh split
        x2 = _r(3, 27, 27, 96, scale=1.0, seed=3)
        w2 = _r(256, 5, 5, 48, scale=0.1, seed=4)
        outs = []
        for var in (4, 8):
            lib.hvk_hc_variant(var)
            y = torch.empty(3, 27, 27, 256, dtype=torch.bfloat16,
                            device="cuda")
            rc = lib.hvk_conv_fwd_hc(
                x2.data_ptr(), w2.data_ptr(), None, y.data_ptr(), 3, 27, 27,
                96, 256, 5, 5, 2, 2, 27, 27, 2, 0, None,
                torch.cuda.current_stream().cuda_stream)
            assert rc == 0, var
            outs.append(y)
        torch.cuda.synchronize()
        _close(outs[1], outs[0], 4e-3)
        # the automatic policy takes AlexNet conv4 and leaves VGG conv2_2
        # (measured slower) to the GEMM
        lib.hvk_hc_variant(-2)
        rc = lib.hvk_conv_fwd_hc(
            x.data_ptr(), w.data_ptr(), None, ref.data_ptr(), 3, 13, 13, 384,
            384, 3, 3, 1, 1, 13, 13, 2, 0, None,
            torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        xv = _r(1, 112, 112, 128, scale=1.0, seed=5)
        wv = _r(128, 3, 3, 128, scale=0.1, seed=6)
        yv = torch.empty(1, 112, 112, 128, dtype=torch.bfloat16,
                         device="cuda")
        rc = lib.hvk_conv_fwd_hc(
            xv.data_ptr(), wv.data_ptr(), None, yv.data_ptr(), 1, 112, 112,
            128, 128, 3, 3, 1, 1, 112, 112, 1, 0, None,
            torch.cuda.current_stream().cuda_stream)
        assert rc == -2
        # a configuration for another kernel size is not taken
        lib.hvk_hc_variant(4)
        rc = lib.hvk_conv_fwd_hc(
            x.data_ptr(), w.data_ptr(), None, ref.data_ptr(), 3, 13, 13, 384,
            384, 3, 3, 1, 1, 13, 13, 2, 0, None,
            torch.cuda.current_stream().cuda_stream)
        assert rc == -2
    finally:
        lib.hvk_hc_variant(-2)
        lib.hvk_hc32(1)


# conv_hc32 (32x32x16 MFMA, one tap per k-step) against the float32
# reference and against the 16x16x32 configurations (hvk_hc32(0)), forced on
# every shape it supports (variant -1), at AlexNet and VGG-16 geometries:
# the 224-wide window of conv1_2 and the 56 / 28 / 14-wide layers, forward
# and backward-data (the VGG backward-data shapes and the
# 224-wide window had no pinned result)
HC32 = [
    # kind, N, H, W, C, OC, K, pad, groups
    ("fwd", 3, 13, 13, 256, 384, 3, 1, 1),       # AlexNet conv3: 512 x 128
    ("fwd", 3, 13, 13, 384, 384, 3, 1, 2),       # conv4: 512 x 96
    ("fwd", 64, 13, 13, 384, 256, 3, 1, 2),      # conv5, several items / WG
    ("dgrad", 3, 13, 13, 256, 384, 3, 1, 1),     # conv3 dgrad
    ("dgrad", 40, 13, 13, 384, 384, 3, 1, 2),    # conv4 dgrad
    ("dgrad", 3, 13, 13, 384, 256, 3, 1, 2),     # conv5 dgrad
    ("fwd", 1, 224, 224, 64, 64, 3, 1, 1),       # VGG conv1_2
    ("dgrad", 1, 224, 224, 64, 64, 3, 1, 1),
    ("fwd", 2, 56, 56, 256, 256, 3, 1, 1),       # VGG conv3_2
    ("dgrad", 2, 56, 56, 256, 256, 3, 1, 1),
    ("fwd", 2, 28, 28, 512, 512, 3, 1, 1),       # VGG conv4_2
    ("dgrad", 2, 28, 28, 512, 512, 3, 1, 1),
    ("fwd", 3, 14, 14, 512, 512, 3, 1, 1),       # VGG conv5_2
    ("dgrad", 3, 14, 14, 512, 512, 3, 1, 1),
    # the 5 x 5 tile (configuration 24: 512 x 64, window pitch OW + 4):
    # AlexNet conv2 forward, and several items per workgroup
    ("fwd", 3, 27, 27, 96, 256, 5, 2, 2),
    ("fwd", 40, 27, 27, 96, 256, 5, 2, 2),
]


@pytest.mark.parametrize("case", HC32)
def test_conv_hc32_matches_reference_and_hc16(case):
    kind, N, H, W, C, OC, K, pad, g = case
    x = _r(N, H, W, C, scale=2.0, seed=11)
    w = _r(OC, K, K, C // g, scale=0.2, seed=12)
    b = torch.randn(OC, device="cuda") * 0.1
    dy = _r(N, H, W, OC, scale=1.0, seed=13)

    def run():
        if kind == "fwd":
            return ops.conv_fwd(x, w, b, (1, 1), (pad,) * 4, g, act="str")
        return ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), (pad,) * 4, g,
                              aux=x, aux_act="str")
    prev = ops._CONV_HC
    out = {}
    try:
        ops.set_conv_hc(True, -1)
        for m32 in (True, False):
            ops.set_conv_hc32(m32)
            out[m32] = run()
            torch.cuda.synchronize()
            var = ops.conv_hc_last_variant()
            assert (var >= 21) == m32, (m32, var)
    finally:
        ops.set_conv_hc32(True)
        ops.set_conv_hc(prev, -2)
    if kind == "fwd":
        ref = F.conv2d(F.pad(x.permute(0, 3, 1, 2).float(), (pad,) * 4),
                       w.permute(0, 3, 1, 2).float(), b,
                       groups=g).clamp_min(0).permute(0, 2, 3, 1)
    else:
        ref = torch.nn.grad.conv2d_input(
            (N, C, H, W), w.permute(0, 3, 1, 2).float(),
            dy.permute(0, 3, 1, 2).float(), padding=pad,
            groups=g).permute(0, 2, 3, 1) * (x.float() > 0)
    _close(out[True], ref, 1e-2)
    _close(out[True], out[False], 1e-2)
    # no bias / no activation path of the forward, and a non-zero bias read
    # from the per-item bias block (tiles of several items per workgroup)
    assert torch.isfinite(out[True].float()).all()


@pytest.mark.parametrize("shape", [
    (3, 13, 13, 256, 384, 3, 1, 1),        # conv3
    (64, 13, 13, 384, 384, 3, 1, 2),       # conv4
    (3, 13, 13, 384, 256, 3, 1, 2),        # conv5
    (2, 27, 27, 96, 256, 5, 2, 2),         # conv2: 16x16 kernel, -3
])
def test_conv_hc32_dgrad_packs_forward_layout_weights(shape):
    """hvk_conv_dgrad_hc_w (the filter bank packed straight from the forward
    weights [OC][KH][KW][Cg]) is bit-identical to hvk_conv_dgrad_hc on the
    permuted [g][c][kh][kw][oc] copy, and declines (-3) the plans that are
    not conv_hc32."""
    from veles_amd.ops import _lib
    lib = _lib.lib()
    N, H, W, C, OC, K, pad, g = shape
    dy = _r(N, H, W, OC, scale=1.0, seed=6)
    w = _r(OC, K, K, C // g, scale=0.2, seed=7)
    aux = _r(N, H, W, C, scale=2.0, seed=8)
    OCg, Cg = OC // g, C // g
    wt = w.view(g, OCg, K, K, Cg).permute(0, 4, 2, 3, 1).contiguous()
    wp = ops._hc_wpack(1, N, H, W, C, OC, K, K, pad, pad, H, W, g, aux, aux,
                       dy.device)
    outs = []
    for fn, ww in ((lib.hvk_conv_dgrad_hc, wt), (lib.hvk_conv_dgrad_hc_w, w)):
        out = torch.empty(N, H, W, C, dtype=torch.bfloat16, device="cuda")
        rc = fn(ops._p(dy), ops._p(ww), ops._p(out), N, H, W, C, OC, K, K,
                pad, pad, H, W, g, ops._p(aux), ops.act_code("str"),
                ops._p(wp), ops._s(dy))
        outs.append((rc, out))
    torch.cuda.synchronize()
    if wp is None:
        assert outs[1][0] == -3 or outs[1][0] == -2
        return
    assert outs[0][0] == 0 and outs[1][0] == 0
    assert torch.equal(outs[0][1], outs[1][1])
