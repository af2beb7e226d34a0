"""HIP kernel numerics: every kernel vs the float32 PyTorch reference of the
same op (the CPU path of veles_amd.ops), plus the NaN-tail overflow guard of
the reference test-suite (veles/tests/doubling_reset.py:41-64)."""
import pytest
import torch

import veles_amd.ops as ops

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


@pytest.fixture(autouse=True, scope="module")
def _gemm_variant():
    """HVK_TEST_GEMM_VARIANT=v runs this module's GEMM / conv kernels on the
    library's A/B schedule v (hvk_set_gemm_variant), default schedule
    otherwise."""
    import os
    v = os.environ.get("HVK_TEST_GEMM_VARIANT")
    if v is None:
        yield
        return
    fn = ops._lib.lib().hvk_set_gemm_variant
    fn(int(v))
    yield
    fn(-1)


def rnd(*shape, scale=1.0, dtype=BF, seed=0):
    g = torch.Generator().manual_seed(seed + sum(shape))
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def close(gpu, ref, tol):
    gpu = gpu.float().cpu()
    ref = ref.float().cpu()
    err = (gpu - ref).abs().max().item()
    mag = ref.abs().max().item() + 1e-6
    assert err <= tol * mag, "max err %g vs scale %g (tol %g)" % (err, mag, tol)


@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(17, 1999, 231), (7, 9, 8), (9, 7, 800),
                                   (1, 1, 1), (256, 384, 512),
                                   (1000, 100, 784), (640, 512, 1000),
                                   (384, 640, 64), (200, 136, 96),
                                   # 96-row tile variant (65..96 rows)
                                   (80, 300, 512), (96, 1024, 256)])
def test_gemm_layouts(ta, tb, M, N, K):
    a = rnd(K, M) if ta else rnd(M, K)
    b = rnd(N, K, seed=1) if tb else rnd(K, N, seed=1)
    ref = ops.gemm(a, b, trans_a=bool(ta), trans_b=bool(tb),
                   out_dtype=torch.float32)
    got = ops.gemm(a.to(DEV), b.to(DEV), trans_a=bool(ta), trans_b=bool(tb),
                   out_dtype=torch.float32)
    torch.cuda.synchronize()
    close(got, ref, 2e-3)


def test_gemm_restrides_unaligned_rows():
    """Operands whose rows miss the 16-B grid (odd pitch, offset views) are
    re-strided before the LDS-DMA kernel: same result as aligned copies."""
    big = rnd(300, 1003)
    a = big[:, 1:1002]          # pointer 2 B off, pitch 1003
    b = rnd(129, 1001, seed=2)  # pitch 1001
    ref = ops.gemm(a.contiguous(), b, trans_b=True, out_dtype=torch.float32)
    got = ops.gemm(big.to(DEV)[:, 1:1002], b.to(DEV), trans_b=True,
                   out_dtype=torch.float32)
    torch.cuda.synchronize()
    close(got, ref, 2e-2)


@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_odd_dims_zero_padded(ta, tb):
    """A large GEMM with odd M / N / K runs on zero-padded operands (the
    LDS-DMA loaders) and matches the fp32 reference, bias included."""
    M, N, K = 331, 257, 1001
    a = rnd(K, M) if ta else rnd(M, K)
    b = rnd(N, K, seed=1) if tb else rnd(K, N, seed=1)
    bias = rnd(N, seed=2, dtype=torch.float32)
    use_bias = bool(tb)  # an MN-major B pads N: no bias then (not padded)
    ref = ops.gemm(a, b, trans_a=bool(ta), trans_b=bool(tb),
                   bias=bias if use_bias else None, act="relu",
                   out_dtype=torch.float32)
    got = ops.gemm(a.to(DEV), b.to(DEV), trans_a=bool(ta), trans_b=bool(tb),
                   bias=bias.to(DEV) if use_bias else None, act="relu",
                   out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert got.shape == (M, N)
    close(got, ref, 2e-2)


def test_gemm_asymmetric_identity():
    # A = I with an asymmetric B catches a transposed C-write
    n = 128
    a = torch.eye(n).to(BF)
    b = (torch.arange(n * n).view(n, n) % 97).float().to(BF)
    got = ops.gemm(a.to(DEV), b.to(DEV), trans_b=False, out_dtype=torch.float32)
    assert torch.equal(got.cpu(), b.float())


@pytest.mark.parametrize("act", ["linear", "tanh", "relu", "strict_relu",
                                 "sigmoid"])
@pytest.mark.parametrize("n", [4096, 1003])
def test_standalone_activation(act, n):
    """Activation units: the bf16 x8 kernels (n % 8 == 0) and the scalar
    kernel (odd n), forward and backward, against the fp32 reference."""
    x = rnd(n, scale=2.0)
    err = rnd(n, seed=5)
    y_ref = ops.act_fwd_ref(x.float(), act)
    y = ops.act_fwd(x.to(DEV), act)
    torch.cuda.synchronize()
    close(y, y_ref, 2e-2)
    yb = y_ref.to(BF)
    d_ref = err.float() * ops.act_bwd_ref(yb.float(), act)
    d = ops.act_bwd(err.to(DEV), yb.to(DEV), act)
    torch.cuda.synchronize()
    close(d, d_ref, 2e-2)


def test_gemm_epilogue_bias_act_aux():
    M, N, K = 300, 260, 192
    a, w = rnd(M, K), rnd(N, K, seed=2)
    bias = torch.randn(N)
    aux = rnd(M, N, seed=3)
    for act in (0, 1, 2, 3, 4):
        ref = ops.gemm(a, w, trans_b=True, bias=bias, act=act, aux=aux,
                       aux_act=3, out_dtype=torch.float32)
        got = ops.gemm(a.to(DEV), w.to(DEV), trans_b=True,
                       bias=bias.to(DEV), act=act, aux=aux.to(DEV),
                       aux_act=3, out_dtype=torch.float32)
        close(got, ref, 5e-3)


@pytest.mark.parametrize("tb", [1, 0])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm_auto_splitk_epilogue(tb, out_dtype):
    """Few output tiles and a long K (the FC layers at batch 512) take the
    split-K path (hvk_gemm_splitk: each K split stores to its own workspace
    slice, one epilogue pass sums them in order): bias, activation and aux
    derivative against fp32, and bit-identical across runs."""
    M, N, K = 256, 1000, 4096
    assert ops.auto_splitk(M, N, K, torch.empty(M, N, device=DEV)) > 1
    a, w = rnd(M, K), rnd(N, K, seed=2) if tb else rnd(K, N, seed=2)
    bias = torch.randn(N)
    aux = rnd(M, N, seed=3)
    for act in (0, 1, 3, 4):
        ref = ops.gemm(a, w, trans_b=bool(tb), bias=bias, act=act, aux=aux,
                       aux_act=3, out_dtype=torch.float32)
        got = ops.gemm(a.to(DEV), w.to(DEV), trans_b=bool(tb),
                       bias=bias.to(DEV), act=act, aux=aux.to(DEV),
                       aux_act=3, out_dtype=out_dtype)
        close(got.float(), ref, 1e-2 if out_dtype == torch.bfloat16 else
              5e-3)
        again = ops.gemm(a.to(DEV), w.to(DEV), trans_b=bool(tb),
                         bias=bias.to(DEV), act=act, aux=aux.to(DEV),
                         aux_act=3, out_dtype=out_dtype)
        assert torch.equal(got, again)


@pytest.mark.parametrize("M,N,K,sk", [(1024, 1000, 4096, 4), (200, 64, 3000, 3),
                                      (130, 136, 1100, 7)])
def test_gemm_splitk_slices(M, N, K, sk):
    """Explicit split counts, including a K that leaves the last split short
    and a split count launch() lowers (7 requested over 1100 -> 6 of 192):
    the finishing pass sums exactly the slices the GEMM wrote."""
    a, w = rnd(M, K), rnd(N, K, seed=5)
    bias = torch.randn(N)
    ref = ops.gemm(a, w, trans_b=True, bias=bias, act=1,
                   out_dtype=torch.float32)
    old = ops._splitk_forced
    ops._splitk_forced = sk
    try:
        got = ops.gemm(a.to(DEV), w.to(DEV), trans_b=True, bias=bias.to(DEV),
                       act=1, out_dtype=torch.float32)
    finally:
        ops._splitk_forced = old
    close(got, ref, 5e-3)


def test_gemm_splitk_accumulate():
    M, N, K = 96, 200, 4096
    a, b = rnd(K, M), rnd(K, N, seed=4)
    ref = ops.gemm(a, b, trans_a=True, accumulate=True)
    out = torch.zeros(M, N, device=DEV)
    ops.gemm(a.to(DEV), b.to(DEV), trans_a=True, out=out, accumulate=True,
             splits=8)
    close(out, ref, 2e-3)


@pytest.mark.parametrize("M,N,K", [(96, 363, 5000), (100, 784, 100),
                                   (256, 128, 64)])
def test_gemm_fused_bias_grad(M, N, K):
    a, b = rnd(K, M), rnd(K, N, seed=6)
    ref = torch.zeros(M, N)
    rbg = torch.zeros(M)
    ops.gemm(a, b, trans_a=True, out=ref, accumulate=True, bias_grad=rbg)
    out = torch.zeros(M, N, device=DEV)
    bg = torch.zeros(M, device=DEV)
    ops.gemm(a.to(DEV), b.to(DEV), trans_a=True, out=out, accumulate=True,
             splits=4, bias_grad=bg)
    close(out, ref, 2e-3)
    close(bg, rbg, 2e-3)


def test_gemm_nan_tail_guard():
    M, N, K = 33, 65, 64
    a, b = rnd(M, K), rnd(N, K, seed=5)
    big = torch.full((2 * M, N), float("nan"), device=DEV)
    ops.gemm(a.to(DEV), b.to(DEV), trans_b=True, out=big[:M],
             out_dtype=torch.float32)
    assert torch.isnan(big[M:]).all()
    assert not torch.isnan(big[:M]).any()


CONVS = [
    # N, H, W, C, OC, KH, KW, sliding(x,y), padding(l,t,r,b), groups
    (2, 13, 13, 16, 24, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (2, 27, 27, 96, 256, 5, 5, (1, 1), (2, 2, 2, 2), 2),
    (2, 35, 35, 3, 96, 11, 11, (4, 4), (0, 0, 0, 0), 1),
    (3, 9, 11, 8, 16, 3, 2, (2, 1), (1, 0, 0, 1), 1),
    (1, 7, 7, 5, 6, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (2, 14, 14, 64, 64, 3, 3, (1, 1), (1, 1, 1, 1), 4),
    # space-to-depth path (C*s*s % 8 == 0) with padding, and the run path
    (2, 40, 37, 3, 64, 8, 8, (4, 4), (2, 1, 2, 1), 1),
    (2, 20, 20, 2, 16, 5, 5, (2, 2), (2, 2, 2, 2), 1),
    (2, 31, 29, 3, 32, 7, 7, (2, 2), (3, 3, 3, 3), 1),
    # direct tiny-reduction forward (LeNet conv1: C = 1, 5 x 5 -> 20; OC 40)
    (2, 28, 28, 1, 20, 5, 5, (1, 1), (0, 0, 0, 0), 1),
    (2, 11, 9, 1, 40, 3, 3, (2, 1), (1, 0, 1, 1), 1),
    # channel-padded path: C = 20 -> 24 (LeNet conv2), C = 3 at stride 1
    (2, 12, 12, 20, 50, 5, 5, (1, 1), (0, 0, 0, 0), 1),
    (2, 16, 16, 3, 64, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    # branch-free DMA addressing paths (gemm.hip kFast loaders): OH*OW < 64
    # (general wgrad loader), 1x1, asymmetric padding with KH != KW,
    # stride-2 dgrad (per-slot path) with OH*OW == 64
    (2, 7, 7, 16, 32, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (3, 10, 12, 128, 64, 1, 1, (1, 1), (0, 0, 0, 0), 1),
    (2, 12, 9, 32, 48, 3, 5, (1, 1), (2, 0, 1, 2), 2),
    (2, 16, 16, 48, 40, 3, 3, (2, 2), (1, 1, 1, 1), 1),
    # LeNet conv2: output channels off the 8-grid (dgrad zero-pads them)
    (4, 12, 12, 20, 50, 5, 5, (1, 1), (0, 0, 0, 0), 1),
]


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd(cfg):
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    x = rnd(N, H, W, C)
    w = rnd(OC, KH, KW, C // g, seed=1, scale=0.1)
    b = torch.randn(OC)
    for act in (0, 3):
        ref = ops.conv_fwd(x, w, b, sl, pad, g, act)
        got = ops.conv_fwd(x.to(DEV), w.to(DEV), b.to(DEV), sl, pad, g, act)
        close(got, ref, 1e-2)


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_dgrad(cfg):
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    w = rnd(OC, KH, KW, C // g, seed=1, scale=0.1)
    OH, OW = ops.conv_out_size(H, W, KH, KW, sl, pad)
    dy = rnd(N, OH, OW, OC, seed=2)
    aux = rnd(N, H, W, C, seed=3)
    ref = ops.conv_dgrad(dy, w, (N, H, W, C), sl, pad, g, aux=aux, aux_act=3)
    got = ops.conv_dgrad(dy.to(DEV), w.to(DEV), (N, H, W, C), sl, pad, g,
                         aux=aux.to(DEV), aux_act=3)
    close(got, ref, 1e-2)


HALO_CONVS = [c for c in CONVS if c[7] == (1, 1)] + [
    # AlexNet conv2 / conv1-after-space-to-depth / conv4 shapes (small batch)
    (2, 27, 27, 96, 256, 5, 5, (1, 1), (2, 2, 2, 2), 2),
    (2, 57, 57, 48, 96, 3, 3, (1, 1), (0, 0, 0, 0), 1),
    (2, 13, 13, 384, 384, 3, 3, (1, 1), (1, 1, 1, 1), 2),
    (3, 20, 23, 64, 40, 3, 3, (1, 1), (1, 1, 1, 1), 1)]


@pytest.mark.parametrize("cfg", HALO_CONVS)
def test_conv_halo_matches_implicit_gemm(cfg):
    """Stride-1 forward / backward-data with the input tile in LDS
    (conv_halo.hip) against the implicit-GEMM kernels: the same products in
    the same MFMA order, so bit-identical outputs (where the halo path does
    not apply it falls back, trivially identical)."""
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    x = rnd(N, H, W, C).to(DEV)
    w = rnd(OC, KH, KW, C // g, seed=1, scale=0.1).to(DEV)
    b = torch.randn(OC).to(DEV)
    OH, OW = ops.conv_out_size(H, W, KH, KW, sl, pad)
    dy = rnd(N, OH, OW, OC, seed=2).to(DEV)
    aux = rnd(N, H, W, C, seed=3).to(DEV)
    res = {}
    lib = ops._lib.lib()
    # -1: f32-staged epilogues, 54: register epilogues (bf16 C image)
    for v in (-1, 54):
        for halo in (False, True):
            ops.set_conv_halo(halo, dgrad=halo)
            try:
                lib.hvk_set_gemm_variant(v)
                y = ops.conv_fwd(x, w, b, sl, pad, g, 3)
                dx = ops.conv_dgrad(dy, w, (N, H, W, C), sl, pad, g, aux=aux,
                                    aux_act=3)
                torch.cuda.synchronize()
            finally:
                lib.hvk_set_gemm_variant(-1)
                ops.set_conv_halo(True, dgrad=False)
            res[(v, halo)] = (y.cpu(), dx.cpu())
    for k in res:
        assert torch.equal(res[(-1, False)][0], res[k][0])
        assert torch.equal(res[(-1, False)][1], res[k][1])


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_wgrad(cfg):
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    x = rnd(N, H, W, C)
    OH, OW = ops.conv_out_size(H, W, KH, KW, sl, pad)
    dy = rnd(N, OH, OW, OC, seed=2)
    ref = torch.zeros(OC, KH, KW, C // g)
    rb = torch.zeros(OC)
    ops.conv_wgrad(x, dy, ref, sl, pad, g, dbias=rb)
    got = torch.zeros(OC, KH, KW, C // g, device=DEV)
    gb = torch.zeros(OC, device=DEV)
    ops.conv_wgrad(x.to(DEV), dy.to(DEV), got, sl, pad, g, dbias=gb)
    close(got, ref, 1e-2)
    close(gb, rb, 1e-2)


@pytest.mark.parametrize("mode", ["max", "avg", "maxabs"])
@pytest.mark.parametrize("shape,k,s", [((2, 55, 55, 96), 3, 2),
                                       ((2, 56, 54, 16), 3, 2),
                                       ((2, 13, 13, 5), 3, 2),
                                       ((1, 8, 8, 16), 2, 2),
                                       # 4- and 2-channel lanes (LeNet)
                                       ((2, 24, 24, 20), 2, 2),
                                       ((2, 8, 8, 50), 2, 2),
                                       ((2, 9, 9, 12), 3, 2),
                                       # AlexNet pool5 (2x2-block backward)
                                       ((2, 13, 13, 256), 3, 2)])
def test_pool(mode, shape, k, s):
    x = rnd(*shape)
    y, am = ops.pool_fwd(x, k, k, (s, s), mode)
    yg, amg = ops.pool_fwd(x.to(DEV), k, k, (s, s), mode)
    close(yg, y, 1e-6)
    if mode != "avg":
        assert torch.equal(amg.cpu().long(), am.long())
    dy = rnd(*y.shape, seed=7)
    aux = rnd(*shape, seed=8)
    dx = ops.pool_bwd(dy, am, shape, k, k, (s, s), mode, aux=aux, aux_act=3)
    dxg = ops.pool_bwd(dy.to(DEV), amg, shape, k, k, (s, s), mode,
                       aux=aux.to(DEV), aux_act=3)
    close(dxg, dx, 1e-2)


@pytest.mark.parametrize("shape", [(3, 13, 13, 256), (2, 14, 12, 24),
                                   (1, 27, 27, 96)])
def test_pool_bwd_block_matches_per_pixel(shape):
    """3x3 / stride-2 max-pool backward: the 2x2-block kernel (each window's
    gradient and argmax loaded once per block) against the per-pixel kernel
    (hvk_set_pool_bwd_variant 1), odd and even image sides, with a fused
    ReLU derivative; the window sums may differ in order only."""
    lib = ops._lib.lib()
    x = rnd(*shape, scale=2.0).to(DEV)
    y, am = ops.pool_fwd(x, 3, 3, (2, 2), "max")
    dy = rnd(*y.shape, seed=7).to(DEV)
    outs = []
    try:
        for v in (1, 0):
            lib.hvk_set_pool_bwd_variant(v)
            outs.append(ops.pool_bwd(dy, am, shape, 3, 3, (2, 2), "max",
                                     aux=x, aux_act=3))
            torch.cuda.synchronize()
    finally:
        lib.hvk_set_pool_bwd_variant(0)
    a, b = outs[0].float().cpu(), outs[1].float().cpu()
    assert torch.allclose(a, b, rtol=1 / 128, atol=0)
    assert b.abs().sum().item() > 0


@pytest.mark.parametrize("C", [96, 256, 13])
def test_lrn(C):
    x = rnd(3, 7, 5, C, scale=3.0)
    y = ops.lrn_fwd(x, 5, 2e-4, 0.75, 2.0)
    close(ops.lrn_fwd(x.to(DEV), 5, 2e-4, 0.75, 2.0), y, 1e-2)
    dy = rnd(3, 7, 5, C, seed=3)
    dx = ops.lrn_bwd(x, dy, 5, 2e-4, 0.75, 2.0)
    close(ops.lrn_bwd(x.to(DEV), dy.to(DEV), 5, 2e-4, 0.75, 2.0), dx, 1e-2)


def test_softmax_ce_and_mse():
    B, C = 37, 1000
    logits = rnd(B, C, scale=3.0, dtype=torch.float32)
    labels = torch.randint(0, C, (B,), dtype=torch.int32)
    labels[5] = -1
    err = torch.empty(B, C)
    m = torch.zeros(3)
    ops.softmax_ce(logits, labels, err=err, metrics=m)
    errg = torch.empty(B, C, device=DEV)
    mg = torch.zeros(3, device=DEV)
    ops.softmax_ce(logits.to(DEV), labels.to(DEV), err=errg, metrics=mg)
    close(errg, err, 1e-4)
    close(mg, m, 1e-4)
    y, t = rnd(9, 33, dtype=torch.float32), rnd(9, 33, seed=1,
                                               dtype=torch.float32)
    e, mm = torch.empty(9, 33), torch.zeros(3)
    ops.mse(y, t, scale=0.5, err=e, metrics=mm, valid_rows=7)
    eg, mmg = torch.empty(9, 33, device=DEV), torch.zeros(3, device=DEV)
    ops.mse(y.to(DEV), t.to(DEV), scale=0.5, err=eg, metrics=mmg,
            valid_rows=7)
    close(eg, e, 1e-5)
    close(mmg, mm, 1e-4)


def test_sgd_and_colsum():
    n = 10007
    w, g, m = torch.randn(n), torch.randn(n), torch.randn(n)
    segs = [(0, 5000, 0.1, 0.01, 0.0, 0.9), (5000, n, 0.2, 0.001, 0.5, 0.5)]
    wg, gg, mg = w.to(DEV), g.to(DEV), m.to(DEV)
    lp = torch.empty(n, dtype=BF, device=DEV)
    ops.sgd_update(w, g, m, segs, gscale=0.5)
    ops.sgd_update(wg, gg, mg, segs, w_lp=lp, gscale=0.5)
    close(wg, w, 1e-6)
    close(mg, m, 1e-6)
    close(lp, w, 1e-2)
    x = rnd(5000, 300)
    close(ops.col_sum(x.to(DEV)), ops.col_sum(x), 1e-4)


@pytest.mark.parametrize("zero", [True, False, 5056])
def test_sgd_zero_tail(zero):
    """zero_grad=True clears the whole gradient after the update, an int
    offset only grad[offset:] (the split-K layers' tail), False nothing."""
    n = 10048
    w, g, m = torch.randn(n), torch.randn(n), torch.randn(n)
    segs = [(0, 5056, 0.1, 0.0, 0.0, 0.9), (5056, n, 0.2, 0.0, 0.0, 0.5)]
    gg = g.to(DEV)
    ops.sgd_update(w.to(DEV), gg, m.to(DEV), segs,
                   w_lp=torch.empty(n, dtype=BF, device=DEV), zero_grad=zero)
    gc = g.clone()
    ops.sgd_update(w, gc, m, segs, zero_grad=zero)
    zf = 0 if zero is True else (n if zero is False else zero)
    assert torch.equal(gg.cpu(), gc)
    assert torch.equal(gc[:zf], g[:zf]) and not gc[zf:].any()


def test_dropout_mask_matches_reference():
    x = torch.randn(12345)
    y = ops.dropout(x, 0.4, 1234)
    yg = ops.dropout(x.to(DEV), 0.4, 1234)
    close(yg, y, 1e-6)


def test_xorshift_bit_exact():
    g = torch.Generator().manual_seed(5)
    st = torch.randint(-2 ** 62, 2 ** 62, (256, 16), generator=g,
                       dtype=torch.int64)
    stg = st.clone().to(DEV)
    out = ops.xorshift1024star(st, 3)
    outg = ops.xorshift1024star(stg, 3)
    assert torch.equal(outg.cpu(), out)
    assert torch.equal(stg.cpu(), st)


def test_fill_minibatch_u8_bf16():
    src = torch.randint(0, 256, (50, 3 * 16 * 16), dtype=torch.uint8)
    lab = torch.randint(0, 10, (50,), dtype=torch.int32)
    sh = torch.randperm(50).to(torch.int32)
    mean = torch.rand(768) * 128
    rd = torch.rand(768) * 0.02
    d = torch.empty(16, 768, dtype=BF)
    lo, io = torch.empty(16, dtype=torch.int32), torch.empty(16, dtype=torch.int32)
    ops.fill_minibatch(src, sh, 3, 11, d, mean=mean, rdisp=rd, labels=lab,
                       labels_out=lo, idx_out=io)
    dg = torch.empty(16, 768, dtype=BF, device=DEV)
    log, iog = torch.empty_like(lo, device=DEV), torch.empty_like(io, device=DEV)
    ops.fill_minibatch(src.to(DEV), sh.to(DEV), 3, 11, dg, mean=mean.to(DEV),
                       rdisp=rd.to(DEV), labels=lab.to(DEV), labels_out=log,
                       idx_out=iog)
    close(dg, d, 1e-2)
    assert torch.equal(log.cpu(), lo) and torch.equal(iog.cpu(), io)


def test_join_and_cast():
    a, b = rnd(7, 5), rnd(7, 9, seed=1)
    close(ops.join([a.to(DEV), b.to(DEV)]), ops.join([a, b]), 0)
    x = torch.randn(1000)
    close(ops.cast(x.to(DEV), BF), ops.cast(x, BF), 0)


def test_conv_im2col_path_fwd_and_wgrad():
    N, H, W, C, OC, k, s = 2, 35, 35, 3, 96, 11, 4
    x = rnd(N, H, W, C)
    w = rnd(OC, k, k, C, seed=1, scale=0.1)
    b = torch.randn(OC)
    ref = ops.conv_fwd(x, w, b, (s, s), (0, 0, 0, 0), 1, 3)
    got = ops.conv_fwd(x.to(DEV), w.to(DEV), b.to(DEV), (s, s), (0, 0, 0, 0),
                       1, 3)
    close(got, ref, 1e-2)
    close(ops.im2col(x.to(DEV), k, k, (s, s), (0, 0, 0, 0)),
          ops.im2col(x, k, k, (s, s), (0, 0, 0, 0)), 0)
    ws = {}
    ops.conv_fwd(x.to(DEV), w.to(DEV), b.to(DEV), (s, s), (0, 0, 0, 0), 1, 3,
                 col_out=ws)
    assert isinstance(ws["col"], ops.S2DImage)  # reused by the wgrad
    OH, OW = ops.conv_out_size(H, W, k, k, (s, s), (0, 0, 0, 0))
    dy = rnd(N, OH, OW, OC, seed=2)
    dref = torch.zeros(OC, k, k, C)
    ops.conv_wgrad(x, dy, dref, (s, s), (0, 0, 0, 0), 1)
    dgot = torch.zeros(OC, k, k, C, device=DEV)
    ops.conv_wgrad(x.to(DEV), dy.to(DEV), dgot, (s, s), (0, 0, 0, 0), 1,
                   col=ws["col"])
    close(dgot, dref, 1e-2)
    # the space-to-depth gradient workspace clears itself in the fold: a
    # second accumulation adds exactly one more gradient
    ops.conv_wgrad(x.to(DEV), dy.to(DEV), dgot, (s, s), (0, 0, 0, 0), 1,
                   col=ws["col"])
    close(dgot, 2 * dref, 1e-2)


@pytest.mark.parametrize("C,R", [(96, 3001), (256, 3001), (8, 3001),
                                 (4096, 1024), (1000 * 8, 37), (520, 5)])
def test_col_sum_vectorised(C, R):
    """narrow (<= 2048 columns: chunk per thread), wide (the FC bias
    gradients: slabs of rows, four loads in flight) and tiny slabs"""
    x = rnd(R, C)
    close(ops.col_sum(x.to(DEV)), ops.col_sum(x), 1e-4)


@pytest.mark.parametrize("max_mb,count", [(8, 6), (7, 7), (5, 3), (1, 1)])
def test_fill_minibatch_odd_sample(max_mb, count):
    """Odd sample size (unaligned rows): the multi-sample row kernel, with a
    minibatch that is not a multiple of its samples per thread and padded
    rows (labels -1, indices -1, data 0)."""
    src = torch.randint(0, 256, (20, 227 * 3), dtype=torch.uint8)
    lab = torch.randint(0, 10, (20,), dtype=torch.int32)
    sh = torch.randperm(20).to(torch.int32)
    mean, rd = torch.rand(681) * 100, torch.rand(681) * 0.01
    d = torch.empty(max_mb, 681, dtype=BF)
    lo = torch.empty(max_mb, dtype=torch.int32)
    io = torch.empty(max_mb, dtype=torch.int32)
    ops.fill_minibatch(src, sh, 2, count, d, mean=mean, rdisp=rd, labels=lab,
                       labels_out=lo, idx_out=io)
    dg = torch.full((max_mb, 681), 7.0, dtype=BF, device=DEV)
    log = torch.empty_like(lo, device=DEV)
    iog = torch.empty_like(io, device=DEV)
    ops.fill_minibatch(src.to(DEV), sh.to(DEV), 2, count, dg,
                       mean=mean.to(DEV), rdisp=rd.to(DEV),
                       labels=lab.to(DEV), labels_out=log, idx_out=iog)
    close(dg, d, 1e-2)
    assert torch.equal(log.cpu(), lo) and torch.equal(iog.cpu(), io)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_solver_kernel(mode):
    n = 4096 + 13
    w0 = torch.randn(n)
    segs = [(0, 2000, 0.1, 1e-3, 0.2, 0.9, mode, 1e-6, 0.95),
            (2000, n, 0.05, 0.0, 0.0, 0.5, mode, 1e-6, 0.9)]
    wc, s1c, s2c = w0.clone(), torch.zeros(n), torch.zeros(n)
    wg, s1g, s2g = w0.to(DEV), torch.zeros(n, device=DEV), \
        torch.zeros(n, device=DEV)
    lp = torch.zeros(n, dtype=BF, device=DEV)
    for it in range(3):
        g = torch.randn(n, generator=torch.Generator().manual_seed(it))
        ops.solver_update(wc, g.clone(), s1c, s2c, segs)
        gg = g.to(DEV)
        ops.solver_update(wg, gg, s1g, s2g, segs, w_lp=lp, zero_grad=True)
        assert float(gg.abs().max()) == 0.0
    close(wg, wc, 1e-5)
    close(s1g, s1c, 1e-5)
    close(lp.float(), wc, 1e-2)



@pytest.mark.parametrize("shape,n", [
    ((2, 55, 55, 96), 5), ((3, 13, 13, 16), 5), ((2, 14, 12, 8), 3),
    ((1, 16, 17, 24), 3), ((2, 27, 27, 256), 5), ((1, 40, 9, 32), 5),
    ((1, 41, 8, 8), 5)])
def test_lrn_pool_fwd_walk_matches_per_output(shape, n):
    """The vertical-walk forward (strips of output rows, the shared input
    row's column max carried, pixel pairs in packed lanes) against the
    per-output kernel: bit-identical outputs and window indices, including
    strips that do not divide OH and windows clipped at the image edge."""
    lib = ops._lib.lib()
    x = rnd(*shape, scale=3.0).to(DEV)
    res = []
    for v in (1, 0, 2, 3, 4):
        lib.hvk_set_lrn_fwd_variant(v)
        N, H, W, C = shape
        OH, OW = ops.pool_out_size(H, W, 3, 3, 2, 2)
        am8 = torch.zeros(N, OH, OW, C, dtype=torch.uint8, device=DEV)
        y8, _ = ops.lrn_pool_fwd(x, n, 1e-4 / n, 0.75, 1.0, 3, 3, (2, 2),
                                 argmax=am8)
        torch.cuda.synchronize()
        res.append((y8.cpu(), am8.cpu()))
    lib.hvk_set_lrn_fwd_variant(0)
    for r in res[1:]:
        assert torch.equal(res[0][0], r[0])
        assert torch.equal(res[0][1], r[1])


@pytest.mark.parametrize("shape,n,aux_mode", [
    ((2, 55, 55, 96), 5, "x"), ((2, 27, 27, 256), 5, "sep"),
    ((2, 14, 12, 8), 3, "none"), ((1, 15, 17, 24), 9, "x"),
    ((1, 9, 9, 512), 5, "sep")])
def test_lrn_pool_bwd_preload_matches_inline(shape, n, aux_mode):
    """The backward with every load of an iteration issued first (clamped
    addresses, absent windows masked) against loads beside their use:
    the same arithmetic, equal up to one bf16 rounding step."""
    lib = ops._lib.lib()
    alpha, beta, k = 1e-4 / n, 0.75, 1.0
    x = rnd(*shape, scale=3.0)
    if aux_mode == "x":
        x = x.clamp_min(0.0)
    xg = x.to(DEV)
    N, H, W, C = shape
    OH, OW = ops.pool_out_size(H, W, 3, 3, 2, 2)
    am8 = torch.zeros(N, OH, OW, C, dtype=torch.uint8, device=DEV)
    y, _ = ops.lrn_pool_fwd(xg, n, alpha, beta, k, 3, 3, (2, 2), argmax=am8)
    dp = rnd(*y.shape, seed=5).to(DEV)
    aux = {"x": xg, "sep": rnd(*shape, seed=6).to(DEV), "none": None}[aux_mode]
    outs = []
    for v in (1, 0):
        lib.hvk_set_lrn_bwd_variant(v)
        outs.append(ops.lrn_pool_bwd(xg, dp, am8, n, alpha, beta, k, 3, 3,
                                     (2, 2), aux=aux,
                                     aux_act=3 if aux is not None else 0))
        torch.cuda.synchronize()
    lib.hvk_set_lrn_bwd_variant(0)
    # the same arithmetic; the two instantiations may contract one product
    # differently (seen: 3 of 50 M elements one bf16 step apart at b1024)
    a, b = outs[0].float().cpu(), outs[1].float().cpu()
    assert torch.allclose(a, b, rtol=1 / 128, atol=0)


def test_pool_lrn_image_chunks_match_whole(monkeypatch):
    """Past 2^31 elements the 2x2 pooling and the one-byte-argmax LRN-pool
    pair run in image chunks (their kernels index with 32-bit offsets): a
    lowered threshold (chunks of 2, 2, 1 images) against the whole-batch
    launch, bitwise, fused ReLU derivative included."""
    x = rnd(5, 27, 27, 96, scale=3.0).clamp_min(0.0).to(DEV)
    N, H, W, C = x.shape
    n, alpha, beta, k = 5, 1e-4 / 5, 0.75, 1.0
    OH, OW = ops.pool_out_size(H, W, 3, 3, 2, 2)

    def run():
        am8 = torch.zeros(N, OH, OW, C, dtype=torch.uint8, device=DEV)
        y, _ = ops.lrn_pool_fwd(x, n, alpha, beta, k, 3, 3, (2, 2),
                                argmax=am8)
        dp = rnd(*y.shape, seed=5).to(DEV)
        dx = ops.lrn_pool_bwd(x, dp, am8, n, alpha, beta, k, 3, 3, (2, 2),
                              aux=x, aux_act=3)
        x2 = x[:, :26, :26].contiguous()
        p2 = ops.pool2_fwd(x2, "max")
        d2 = ops.pool2_bwd(x2, rnd(*p2.shape, seed=9).to(DEV), "max",
                           aux=x2, aux_act=3)
        torch.cuda.synchronize()
        return [t.cpu() for t in (y, am8, dx, p2, d2)]

    whole = run()
    monkeypatch.setattr(ops, "_CHUNK_ELEMS", 2 * H * W * C + 1)
    assert ops._n_chunks(N, H * W * C) == [(0, 2), (2, 4), (4, 5)]
    for a, b in zip(whole, run()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape,stride,n,aux_mode", [
    ((2, 27, 27, 96), 2, 5, "sep"), ((3, 13, 13, 16), 2, 5, "sep"),
    ((2, 55, 55, 96), 2, 5, "sep"), ((2, 55, 55, 96), 2, 5, "x"),
    ((2, 14, 12, 8), 2, 3, "none"), ((1, 16, 17, 24), 2, 9, "x"),
    ((2, 20, 19, 32), 3, 5, "sep"), ((1, 15, 15, 40), 3, 7, "x"),
    # DPP-halo backward: 2 blocks per wave (C = 256), one (C = 512), and
    # the per-thread fallback past 64 chunks (C = 528)
    ((2, 27, 27, 256), 2, 5, "x"), ((1, 9, 9, 512), 2, 5, "sep"),
    ((1, 7, 7, 528), 2, 5, "sep"),
    # row-marching forward: two 64-lane column groups (OW = 66)
    ((1, 11, 133, 16), 2, 5, "x")])
def test_lrn_pool_fused(shape, stride, n, aux_mode):
    """Fused LRN -> 3x3 max pool forward / backward against the fp32
    reference; stride 2 runs the 2x2-block backward kernel, stride 3 the
    per-pixel one; aux_mode "x" hits the aux-is-input (ReLU) shortcut."""
    alpha, beta, k = 1e-4 / n, 0.75, 1.0
    st = (stride, stride)
    x = rnd(*shape, scale=3.0)
    if aux_mode == "x":
        x = x.clamp_min(0.0)
    xg = x.to(DEV)
    y, am = ops.lrn_pool_fwd(xg, n, alpha, beta, k, 3, 3, st)
    yr, amr = ops.lrn_pool_fwd(x, n, alpha, beta, k, 3, 3, st)
    torch.cuda.synchronize()
    close(y, yr, 1e-2)
    # argmax may differ only where two window values tie in fp32 vs bf16
    assert (am.cpu() != amr).float().mean().item() < 1e-3
    if stride == 2:
        # the one-byte window-index format the AlexNet pair uses on the GPU
        am8 = torch.zeros(am.shape, dtype=torch.uint8, device=DEV)
        y8, _ = ops.lrn_pool_fwd(xg, n, alpha, beta, k, 3, 3, st,
                                 argmax=am8)
        torch.cuda.synchronize()
        assert torch.equal(y8, y)
        off8 = ops.window_index_to_offsets(am8, shape, 3, 3, st).cpu()
        assert (off8 != amr).float().mean().item() < 1e-3
        am = am8
    dp = rnd(*y.shape, seed=5)
    if aux_mode == "sep":
        aux, auxg = rnd(*shape, seed=6), None
        auxg = aux.to(DEV)
    elif aux_mode == "x":
        aux, auxg = x, xg
    else:
        aux = auxg = None
    act = 3 if aux is not None else 0
    dx = ops.lrn_pool_bwd(xg, dp.to(DEV), am, n, alpha, beta, k, 3, 3,
                          st, aux=auxg, aux_act=act)
    dxr = ops.lrn_pool_bwd(x, dp, am.cpu(), n, alpha, beta, k, 3, 3, st,
                           aux=aux, aux_act=act)
    torch.cuda.synchronize()
    close(dx, dxr, 2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["max", "avg", "maxabs"])
@pytest.mark.parametrize("aux_mode", ["none", "sep", "x"])
def test_pool2_argmax_free(mode, aux_mode):
    """2 x 2 / stride-2 pooling without an argmax tensor: the backward
    recomputes the window's choice from x (pool2 kernels) - against the
    argmax-based fp32 reference, with and without a fused activation
    derivative (aux separate, or aux == x for ReLU below)."""
    shape = (3, 14, 10, 24)
    x = rnd(*shape, scale=2.0)
    if aux_mode == "x":
        x = x.clamp_min(0.0)
    xg = x.to(DEV)
    y = ops.pool2_fwd(xg, mode)
    yr, am = ops.pool_fwd(x, 2, 2, (2, 2), mode)
    torch.cuda.synchronize()
    close(y, yr, 1e-2)
    dy = rnd(*y.shape, seed=4)
    aux = auxg = None
    if aux_mode == "sep":
        aux = rnd(*shape, seed=6)
        auxg = aux.to(DEV)
    elif aux_mode == "x":
        aux, auxg = x, xg
    act = 3 if aux is not None else 0
    dx = ops.pool2_bwd(xg, dy.to(DEV), mode, aux=auxg, aux_act=act)
    dxr = ops.pool_bwd(dy, am, shape, 2, 2, (2, 2), mode, aux=aux,
                       aux_act=act)
    torch.cuda.synchronize()
    close(dx, dxr, 1e-2)


# ------------------------------------------ input-derivative activations
@pytest.mark.parametrize("kind,p", [("log", 0.0), ("tanhlog", 0.9),
                                    ("sincos", 0.0), ("mul", 1.7)])
@pytest.mark.parametrize("shape", [(4, 64), (3, 5, 7)])  # vector / scalar
def test_xact(kind, p, shape):
    x = rnd(*shape, scale=2.0)
    e = rnd(*shape, seed=3)
    y = ops.xact(x.to(DEV), kind, p)
    d = ops.xact(x.to(DEV), kind, p, err=e.to(DEV))
    torch.cuda.synchronize()
    close(y, ops.xact_ref(x, kind, p), 1e-2)
    close(d, ops.xact_ref(x, kind, p, bwd=True, err=e), 1e-2)


def test_gather():
    x = rnd(5, 7, 9)
    idx = torch.randint(-1, x.numel(), (3, 11), dtype=torch.int32)
    g = ops.gather(x.to(DEV), idx.to(DEV))
    torch.cuda.synchronize()
    assert torch.equal(g.cpu(), ops.gather(x, idx))


@pytest.mark.parametrize("shape,k,s", [((2, 9, 10, 16), 3, 2),
                                       ((3, 8, 8, 5), 2, 2),
                                       ((1, 7, 5, 3), 3, 3)])
@pytest.mark.parametrize("use_abs", [False, True])
@pytest.mark.parametrize("train", [True, False])
def test_stochastic_pool(shape, k, s, use_abs, train):
    x = rnd(*shape)
    seed = torch.tensor([12345], dtype=torch.int32)
    y, am = ops.stochastic_pool(x.to(DEV), k, k, (s, s), use_abs, train,
                                seed_dev=seed.to(DEV))
    yr, amr = ops.stochastic_pool(x, k, k, (s, s), use_abs, train, seed=12345)
    torch.cuda.synchronize()
    # the draw agrees except where a cumulative probability sits on u
    assert (am.cpu() != amr).float().mean().item() < 2e-3
    same = am.cpu() == amr
    close(y.cpu()[same], yr[same], 1e-2)
    if train:  # a drawn value is the input at the drawn offset
        assert torch.equal(y.cpu().view(-1),
                           x.view(-1)[am.cpu().view(-1).long()])


def test_depooling_scatter_is_pool_backward():
    """Depooling (scatter-add of pooled values to the argmax offsets) runs
    as the max-pooling backward gather; compare with a plain index_put."""
    x = rnd(2, 9, 9, 8)
    y, am = ops.pool_fwd(x.to(DEV), 3, 3, (2, 2), "max")
    v = rnd(*y.shape, seed=4)
    out = ops.pool_bwd(v.to(DEV), am, x.shape, 3, 3, (2, 2), "max")
    ref = torch.zeros(x.numel())
    ref.index_put_((am.cpu().reshape(-1).long(),), v.float().reshape(-1),
                   accumulate=True)
    torch.cuda.synchronize()
    close(out, ref.view(x.shape), 1e-2)


@pytest.mark.parametrize("shape,k,pad", [((3, 227, 227, 3), 11, (0, 0, 0, 0)),
                                         ((1, 35, 33, 3), 11, (2, 1, 2, 1)),
                                         ((2, 19, 21, 3), 8, (3, 2, 0, 0))])
def test_space_to_depth(shape, k, pad):
    """Row-staged space-to-depth (s = 4, C = 3) against a padded view."""
    x = rnd(*shape)
    y = ops.space_to_depth(x.to(DEV), 4, k, k, pad)
    torch.cuda.synchronize()
    N, H, W, C = shape
    _, H2, W2, C2 = y.shape
    pl, pt = pad[0], pad[1]
    xp = torch.zeros(N, H2 * 4, W2 * 4, C, dtype=x.dtype)
    h1, w1 = min(H, H2 * 4 - pt), min(W, W2 * 4 - pl)
    xp[:, pt:pt + h1, pl:pl + w1] = x[:, :h1, :w1]
    ref = xp.view(N, H2, 4, W2, 4, C).permute(0, 1, 3, 2, 4, 5).reshape(
        N, H2, W2, 16 * C)
    assert torch.equal(y.cpu(), ref)


@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("with_bias", [False, True])
def test_gemm_overwrite_gradient(splits, with_bias):
    """accumulate="overwrite": the weight-gradient GEMM writes (and the
    fused bias-gradient column stores) instead of adding - whatever the
    buffers held before; split-K zeroes first."""
    M, N, K = 200, 136, 1024
    a, b = rnd(K, M), rnd(K, N, seed=1)
    out = torch.full((M, N), 7.0, device=DEV)
    bg = torch.full((M,), -3.0, device=DEV) if with_bias else None
    ops.gemm(a.to(DEV), b.to(DEV), trans_a=True, out=out,
             accumulate="overwrite", splits=splits, bias_grad=bg)
    torch.cuda.synchronize()
    ref = a.float().t() @ b.float()
    close(out, ref, 1e-2)
    if with_bias:
        close(bg, a.float().sum(0), 1e-2)
