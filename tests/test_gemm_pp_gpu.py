"""The ping-pong 256 x 128 GEMM main loop (csrc/kernels/gemm_pp.h) against the
128-row loop on large dense NT / NN GEMMs and a split-K accumulation, and
against the float32 reference of the same op.

Both main loops accumulate every output over the same 16x16x32 MFMAs in the
same K order (K tile by K tile, the two 32-deep halves in order), so without
split-K their outputs must be bit-identical.  hvk_set_gemm_variant(30) turns
the ping-pong loop off.  The
shapes are large enough for the launch policy to pick the ping-pong loop
(>= 256 tiles of 256 x 128) and cover partial row / column tiles, a K tail
and the one- and two-K-tile prologues."""
import pytest
import torch

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


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 512), (4100, 4100, 200),
                                   (4096, 4000, 8), (4200, 4096, 72),
                                   (8192, 2048, 1000)])
def test_pp_dense_nt(M, N, K):
    a = rnd(M, K, seed=1)
    b = rnd(N, K, seed=2)
    bias = torch.randn(N, device=DEV)
    old, new = run_variants(lambda: ops.gemm(a, b, trans_b=True, bias=bias,
                                             out_dtype=torch.bfloat16),
                            (30, -1))
    assert torch.equal(old, new)
    close(new, a.float() @ b.float().t() + bias, 1e-2)


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 1024), (2048, 9216, 4096)])
def test_pp_dense_nn(M, N, K):
    """NN (fc backward-data): the MN-major B through transposed reads"""
    a = rnd(M, K, seed=6)
    b = rnd(K, N, seed=7)
    old, new = run_variants(lambda: ops.gemm(a, b, out_dtype=torch.float32),
                            (30, -1))
    assert torch.equal(old, new)
    close(new, a.float() @ b.float(), 1e-2)


def test_pp_splitk_accumulate():
    """split-K f32 accumulation: re-split for the 256-row tiles, staged
    coalesced atomics"""
    M, N, K = 1024, 4096, 9216
    a = rnd(M, K, seed=3)
    b = rnd(N, K, seed=4)

    def run():
        out = torch.full((M, N), 0.5, device=DEV)
        return ops.gemm(a, b, trans_b=True, out=out, accumulate=True,
                        splits=4)
    old, new = run_variants(run, (30, -1))
    ref = a.float() @ b.float().t() + 0.5
    close(old, ref, 1e-3)
    close(new, ref, 1e-3)


def _conv_case(N, H, W, C, OC, k, p, g):
    x = rnd(N, H, W, C, seed=3)
    w = rnd(OC, k, k, C // g, seed=4, scale=0.05)
    return x, w


@pytest.mark.parametrize("cfg", [
    # AlexNet conv2 backward-data (48 channels per group: VAR 4), conv4 /
    # conv5 backward-data and conv4 forward (192 per group -> 3 x 64: VAR 3)
    (128, 27, 27, 96, 256, 5, 2, 2),
    (256, 13, 13, 384, 384, 3, 1, 2),
    (256, 13, 13, 384, 256, 3, 1, 2)])
def test_256_row_narrow_tiles(cfg):
    """the 256-row x 64 tile of gemm_kernel (VAR 3 / 4) against the 128-row
    tile (hvk_set_gemm_variant 40): bit-identical, and against fp32"""
    import torch.nn.functional as F
    N, H, W, C, OC, k, p, g = cfg
    x, w = _conv_case(*cfg)
    pad = (p, p, p, p)
    dy = rnd(N, H, W, OC, seed=5)
    old, new = run_variants(lambda: ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1),
                                                   pad, g), (40, -1))
    assert torch.equal(old, new)
    ref = torch.nn.grad.conv2d_input(
        (N, C, H, W), w.float().permute(0, 3, 1, 2),
        dy.float().permute(0, 3, 1, 2), padding=p,
        groups=g).permute(0, 2, 3, 1)
    close(new, ref, 1e-2)
    b = torch.randn(OC, device=DEV)
    old, new = run_variants(lambda: ops.conv_fwd(x, w, b, (1, 1), pad, g, 3),
                            (40, -1))
    assert torch.equal(old, new)
    ref = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2),
                          w.float().permute(0, 3, 1, 2), b, padding=p,
                          groups=g)).permute(0, 2, 3, 1)
    close(new, ref, 1e-2)


@pytest.mark.parametrize("M,N,K,mode,splits", [
    (4096, 4096, 256, "overwrite", 1),     # fc7-like weight gradient
    (4096, 4352, 520, True, 1),            # partial K tile, accumulate
    (4096, 4096, 4096, True, 4),           # split-K f32 atomics (re-split)
    (4000, 4104, 96, "overwrite", 1)])     # partial row / column tiles
def test_pp256_tn_weight_gradient(M, N, K, mode, splits):
    """TN GEMMs without a bias-gradient column (FC weight gradients with
    engine.fc_bias_colsum) take the 256 x 256 loop with both operands
    MN-major; hvk_gemm_variant 64 keeps the 128-row loop.  Same K order
    without split-K: bit-identical; with split-K: the atomics' order."""
    a = rnd(K, M, seed=3)
    b = rnd(K, N, seed=4)
    init = torch.randn(M, N, device=DEV)

    def run():
        out = init.clone()
        ops.gemm(a, b, trans_a=True, out=out, accumulate=mode, splits=splits)
        return out
    old, new = run_variants(run, (64, -1))
    ref = a.float().t() @ b.float() + (0 if mode == "overwrite" else init)
    if splits == 1:
        assert torch.equal(old, new)
    close(new, ref, 1e-3)
