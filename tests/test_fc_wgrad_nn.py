"""FC weight gradient through dY^T (ops.transpose_colsum) and the NN GEMM
(models/gd.py ``_wgrad_nn``) against the TN GEMM with the fused bias column
and an fp32 torch reference."""
import pytest
import torch

from veles_amd import ops


def test_transpose_colsum_cpu():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(128, 192, generator=g)
    cs = torch.full((192,), 2.0)
    t = ops.transpose_colsum(x, colsum=cs, accumulate=True)
    assert torch.equal(t, x.t())
    torch.testing.assert_close(cs, 2.0 + x.sum(0))


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(64, 64), (3072, 4096), (192, 1024)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_transpose_colsum_gpu(R, C, accumulate):
    g = torch.Generator(device="cuda").manual_seed(R + C)
    x = torch.randn(R, C, generator=g, device="cuda").to(torch.bfloat16)
    cs0 = torch.randn(C, generator=g, device="cuda")
    cs = cs0.clone()
    t = ops.transpose_colsum(x, colsum=cs, accumulate=accumulate)
    torch.cuda.synchronize()
    assert torch.equal(t, x.t().contiguous())   # a pure move: bit-exact
    ref = x.float().sum(0) + (cs0 if accumulate else 0)
    torch.testing.assert_close(cs, ref, rtol=1e-5, atol=1e-4)
    # deterministic: the same sums twice
    cs2 = cs0.clone()
    ops.transpose_colsum(x, colsum=cs2, accumulate=accumulate)
    assert torch.equal(cs, cs2)


@pytest.mark.gpu
def test_transpose_colsum_rejects_ragged_shapes():
    x = torch.zeros(100, 64, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.transpose_colsum(x)


@pytest.mark.gpu
@pytest.mark.parametrize("B,nin,nout", [(256, 1024, 512), (3072, 4096, 1024)])
def test_fc_wgrad_nn_matches_tn_and_fp32(B, nin, nout):
    """The GD path's two forms of dW = dY^T x, db = colsum(dY) against the
    fp32 product of the same bf16 operands (same bf16 K-reduction floor)."""
    g = torch.Generator(device="cuda").manual_seed(B)
    x = torch.randn(B, nin, generator=g, device="cuda").to(torch.bfloat16)
    e = torch.randn(B, nout, generator=g, device="cuda").to(torch.bfloat16)
    ref_w = e.float().t() @ x.float()
    ref_b = e.float().sum(0)
    w_tn = torch.empty(nout, nin, device="cuda")
    b_tn = torch.empty(nout, device="cuda")
    ops.gemm(e, x, trans_a=True, out=w_tn, accumulate="overwrite",
             bias_grad=b_tn)
    w_nn = torch.empty(nout, nin, device="cuda")
    b_nn = torch.empty(nout, device="cuda")
    et = ops.transpose_colsum(e, colsum=b_nn)
    ops.gemm(et, x, out=w_nn, accumulate="overwrite")
    torch.cuda.synchronize()

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    assert rel(w_nn, ref_w) < 1e-5 and rel(w_tn, ref_w) < 1e-5
    assert rel(b_nn, ref_b) < 1e-5 and rel(b_tn, ref_b) < 1e-5
