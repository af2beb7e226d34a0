"""The 256 x 128 / 192 x 128 two-workgroups-per-CU convolution loop
(csrc/kernels/gemm_t4.h) against the 128-row loop and against the float32
reference of the same op.

Both loops accumulate every output over the same 16x16x32 MFMAs in the same K
order, so without split-K the forward and backward-data outputs must be
bit-identical.  hvk_set_gemm_variant(50) turns the T4 loop off, 53 runs it
with the direct (register -> global) epilogue and 54 with the register
epilogue (bf16 C image) instead of the default f32-staged one; 51 / 52 force
its first / second orientation (forward and backward-data: P = pixels (256)
or P = channels (192, transposed epilogue); weight gradient: P = im2col
columns (256, transposed) or P = output channels (192)).  The shapes are the
AlexNet / VGG layers at small batches, with partial row tiles, K tails and
grouped convolutions."""
import pytest
import torch
import torch.nn.functional as F

import veles_amd.ops as ops

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.rand(*shape, generator=g, device=DEV) * 2 - 1).mul_(
        scale).to(BF)


def run_variants(fn, variants):
    lib = ops._lib.lib()
    out = []
    try:
        for v in variants:
            lib.hvk_set_gemm_variant(v)
            out.append(fn().clone())
    finally:
        lib.hvk_set_gemm_variant(-1)
    torch.cuda.synchronize()
    return out


def close(got, ref, tol):
    err = (got.float() - ref.float()).abs().max().item()
    mag = ref.float().abs().max().item() + 1e-6
    assert err <= tol * mag, "max err %g vs scale %g" % (err, mag)


def nchw(t):
    return t.float().permute(0, 3, 1, 2)


CASES = [
    # N, H, W, C, OC, k, pad, groups
    (3, 27, 27, 96, 256, 5, 2, 2),      # AlexNet conv2 (128 per group)
    (5, 13, 13, 256, 384, 3, 1, 1),     # conv3 (N = 384, dgrad N = 256)
    (7, 13, 13, 384, 384, 3, 1, 2),     # conv4 (192 per group)
    (6, 13, 13, 384, 256, 3, 1, 2),     # conv5 (128 out, 192 in per group)
    (2, 28, 28, 128, 256, 3, 1, 1),     # VGG-like
]


@pytest.mark.parametrize("cfg", CASES)
@pytest.mark.parametrize("force", [-1, 51, 52, 53, 54])
def test_t4_conv_fwd(cfg, force):
    N, H, W, C, OC, k, p, g = cfg
    x = rnd(N, H, W, C, seed=1)
    w = rnd(OC, k, k, C // g, seed=2, scale=0.05)
    b = torch.randn(OC, device=DEV)
    pad = (p, p, p, p)
    old, new = run_variants(lambda: ops.conv_fwd(x, w, b, (1, 1), pad, g, 3),
                            (50, force))
    assert torch.equal(old, new)
    ref = F.relu(F.conv2d(nchw(x), nchw(w), b, padding=p,
                          groups=g)).permute(0, 2, 3, 1)
    close(new, ref, 1e-2)


@pytest.mark.parametrize("cfg", CASES)
@pytest.mark.parametrize("force", [-1, 51, 52, 53, 54])
def test_t4_conv_dgrad(cfg, force):
    N, H, W, C, OC, k, p, g = cfg
    w = rnd(OC, k, k, C // g, seed=4, scale=0.05)
    dy = rnd(N, H, W, OC, seed=5)
    aux = rnd(N, H, W, C, seed=6)   # ReLU derivative of the layer below
    pad = (p, p, p, p)

    def run():
        return ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), pad, g, aux=aux,
                              aux_act=3)
    old, new = run_variants(run, (50, force))
    assert torch.equal(old, new)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), nchw(w), nchw(dy),
                                     padding=p, groups=g).permute(0, 2, 3, 1)
    ref = ref * (aux.float() > 0).float()
    close(new, ref, 1e-2)


@pytest.mark.parametrize("cfg", CASES)
@pytest.mark.parametrize("force", [-1, 51, 52, 53, 54])
@pytest.mark.parametrize("splits", [1, 5])
def test_t4_conv_wgrad(cfg, force, splits):
    """accumulating weight gradient + fused bias gradient; split-K through
    f32 atomics is not bit-identical, unsplit read-modify-write is"""
    N, H, W, C, OC, k, p, g = cfg
    x = rnd(N, H, W, C, seed=7)
    dy = rnd(N, H, W, OC, seed=8)
    pad = (p, p, p, p)

    def run():
        dw = torch.full((OC, k, k, C // g), 0.25, device=DEV)
        db = torch.full((OC,), 0.5, device=DEV)
        ops.conv_wgrad(x, dy, dw, (1, 1), pad, g, splits=splits, dbias=db)
        return torch.cat([dw.reshape(-1), db])
    old, new = run_variants(run, (50, force))
    if splits == 1:
        assert torch.equal(old, new)
    ref_w = torch.nn.grad.conv2d_weight(nchw(x), (OC, C // g, k, k),
                                        nchw(dy), padding=p,
                                        groups=g).permute(0, 2, 3, 1) + 0.25
    ref_b = dy.float().reshape(-1, OC).sum(0) + 0.5
    ref = torch.cat([ref_w.reshape(-1), ref_b])
    close(new, ref, 2e-3)
    close(old, ref, 2e-3)


PP_CASES = [
    # N, H, W, C, OC, k, pad, groups: >= 256 outputs per group (forward) /
    # inputs per group (backward-data), partial 256-row tiles, K tails
    (2, 14, 14, 256, 256, 3, 1, 1),
    (3, 13, 13, 384, 256, 3, 1, 1),     # AlexNet conv3 backward-data
    (2, 7, 7, 512, 512, 3, 1, 2),       # 256 per group
    (1, 28, 28, 128, 512, 3, 1, 1),     # forward only: C = 128
]


@pytest.mark.parametrize("cfg", PP_CASES)
def test_pp256_conv_fwd_dgrad(cfg):
    """The 256 x 256 ping-pong loop with the implicit-GEMM loaders
    (hvk_set_gemm_variant(56) forces it for >= 256 outputs per group; the
    default takes it where it fills the CUs) against the 128-row loop:
    bit-identical, and against the float32 reference"""
    N, H, W, C, OC, k, p, g = cfg
    pad = (p, p, p, p)
    x = rnd(N, H, W, C, seed=11)
    w = rnd(OC, k, k, C // g, seed=12, scale=0.05)
    b = torch.randn(OC, device=DEV)
    old, new = run_variants(lambda: ops.conv_fwd(x, w, b, (1, 1), pad, g, 3),
                            (50, 56))
    assert torch.equal(old, new)
    ref = F.relu(F.conv2d(nchw(x), nchw(w), b, padding=p,
                          groups=g)).permute(0, 2, 3, 1)
    close(new, ref, 1e-2)
    if C // g < 256:
        return
    dy = rnd(N, H, W, OC, seed=13)
    aux = rnd(N, H, W, C, seed=14)

    def run():
        return ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), pad, g, aux=aux,
                              aux_act=3)
    old, new = run_variants(run, (50, 56))
    assert torch.equal(old, new)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), nchw(w), nchw(dy),
                                     padding=p, groups=g).permute(0, 2, 3, 1)
    close(new, ref * (aux.float() > 0).float(), 1e-2)


T4_64_CASES = [
    # N, H, W, C, OC, k, pad, groups: 33-64 outputs (forward) / inputs
    # (backward-data) per group - the stacked-wave 256 x 64 T4 tiles
    (3, 27, 27, 96, 256, 5, 2, 2),      # AlexNet conv2 backward-data (48)
    (2, 30, 30, 64, 64, 3, 1, 1),       # VGG conv1_2 (64), partial tiles
    (2, 14, 14, 128, 48, 3, 1, 1),      # forward with 48 outputs
]


@pytest.mark.parametrize("cfg", T4_64_CASES)
def test_t4_64_conv_fwd_dgrad(cfg):
    """hvk_set_gemm_variant(58) selects the (opt-in) 256 x 64 T4 tiles;
    against the 128-row loop (50): bit-identical, and the float32
    reference"""
    N, H, W, C, OC, k, p, g = cfg
    pad = (p, p, p, p)
    x = rnd(N, H, W, C, seed=21)
    w = rnd(OC, k, k, C // g, seed=22, scale=0.05)
    b = torch.randn(OC, device=DEV)
    old, new = run_variants(lambda: ops.conv_fwd(x, w, b, (1, 1), pad, g, 3),
                            (50, 58))
    assert torch.equal(old, new)
    ref = F.relu(F.conv2d(nchw(x), nchw(w), b, padding=p,
                          groups=g)).permute(0, 2, 3, 1)
    close(new, ref, 1e-2)
    dy = rnd(N, H, W, OC, seed=23)
    aux = rnd(N, H, W, C, seed=24)

    def run():
        return ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), pad, g, aux=aux,
                              aux_act=3)
    old, new = run_variants(run, (50, 58))
    assert torch.equal(old, new)
    ref = torch.nn.grad.conv2d_input((N, C, H, W), nchw(w), nchw(dy),
                                     padding=p, groups=g).permute(0, 2, 3, 1)
    close(new, ref * (aux.float() > 0).float(), 1e-2)


@pytest.mark.parametrize("cfg", [
    (2, 14, 14, 256, 256, 3, 1, 1),
    (4, 13, 13, 384, 256, 3, 1, 1),     # KK = 3456 + bias column
    (2, 9, 9, 512, 512, 3, 1, 2),       # 256 per group
])
@pytest.mark.parametrize("splits", [1, 4])
def test_pp256_conv_wgrad(cfg, splits):
    """weight gradient (+ fused bias gradient) on the 256 x 256 ping-pong
    loop with the MN-major dY / im2col loaders (hvk_set_gemm_variant(63))
    against the 128-row loop and the float32 reference (f32 atomics: not
    bit-identical)"""
    N, H, W, C, OC, k, p, g = cfg
    x = rnd(N, H, W, C, seed=31)
    dy = rnd(N, H, W, OC, seed=32)
    pad = (p, p, p, p)

    def run():
        dw = torch.full((OC, k, k, C // g), 0.25, device=DEV)
        db = torch.full((OC,), 0.5, device=DEV)
        ops.conv_wgrad(x, dy, dw, (1, 1), pad, g, splits=splits, dbias=db)
        return torch.cat([dw.reshape(-1), db])
    old, new = run_variants(run, (50, 63))
    ref_w = torch.nn.grad.conv2d_weight(nchw(x), (OC, C // g, k, k),
                                        nchw(dy), padding=p,
                                        groups=g).permute(0, 2, 3, 1) + 0.25
    ref_b = dy.float().reshape(-1, OC).sum(0) + 0.5
    ref = torch.cat([ref_w.reshape(-1), ref_b])
    close(new, ref, 2e-3)
    close(old, ref, 2e-3)
