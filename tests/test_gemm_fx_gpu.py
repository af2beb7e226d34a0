"""Exact-precision SGEMM / DGEMM (csrc/kernels/gemm_f32.hip) and the
reference's precision levels (veles/tests/test_ocl_blas.py:48-110 shapes,
checked against float64 on the host)."""
import pytest
import torch

import veles_amd.ops as ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [(17, 1999, 231), (7, 9, 8), (9, 7, 800), (1, 1, 1), (7777, 17, 219),
          (1777, 1999, 2119)]


def _ref(a, b, ta, tb):
    A = a.double().t() if ta else a.double()
    B = b.double().t() if tb else b.double()
    return A @ B


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_gemm_fx_layouts(dtype, M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.rand(*((K, M) if ta else (M, K)), generator=g,
                   dtype=torch.float64) - 0.5
    b = torch.rand(*((N, K) if tb else (K, N)), generator=g,
                   dtype=torch.float64) - 0.5
    ref = _ref(a, b, ta, tb)
    got = ops.gemm(a.to(DEV, dtype), b.to(DEV, dtype), trans_a=bool(ta),
                   trans_b=bool(tb), out_dtype=dtype)
    torch.cuda.synchronize()
    err = (got.double().cpu() - ref).abs().max().item()
    tol = (1e-4 if dtype == torch.float32 else 1e-12) * max(1.0, K ** 0.5)
    assert err < tol, err


def test_gemm_fx_alpha_beta():
    a = torch.randn(300, 200, dtype=torch.float64)
    b = torch.randn(200, 100, dtype=torch.float64)
    c = torch.randn(300, 100, dtype=torch.float64)
    out = c.to(DEV)
    ops.gemm(a.to(DEV), b.to(DEV), out=out, alpha=0.5, beta=2.0)
    ref = 0.5 * (a @ b) + 2.0 * c
    assert (out.cpu() - ref).abs().max().item() < 1e-10


@pytest.mark.parametrize("level", [1, 2])
def test_precision_levels_reduce_error(level):
    # long dot products with a large common offset: the plain f32 chain
    # loses digits, the compensated tile sums keep them
    K = 1 << 17
    g = torch.Generator().manual_seed(3)
    a = (torch.rand(64, K, generator=g, dtype=torch.float64) + 1.0)
    b = (torch.rand(K, 64, generator=g, dtype=torch.float64) + 1.0)
    ref = a @ b
    ad, bd = a.to(DEV, torch.float32), b.to(DEV, torch.float32)
    # compare against the product of the ROUNDED inputs
    ref = ad.double().cpu() @ bd.double().cpu()
    e0 = (ops.gemm(ad, bd, precision_level=0).double().cpu() - ref).abs().max()
    el = (ops.gemm(ad, bd, precision_level=level).double().cpu() - ref) \
        .abs().max()
    assert el.item() < 0.5 * e0.item(), (e0.item(), el.item())
