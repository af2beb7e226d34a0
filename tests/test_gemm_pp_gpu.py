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
