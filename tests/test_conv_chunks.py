"""Image-chunked convolutions (ops._image_chunks): operands past the 32-bit
buffer offsets of the LDS-DMA loaders run as several launches over image
ranges.  The GPU tests lower the threshold so small tensors take the chunked
route and compare it with the unchunked call: forward and backward-data are
bit-identical (every output element keeps its K order), the weight
gradients accumulate over the chunks (f32 atomics: tolerance)."""
import pytest
import torch

from veles_amd import ops
from veles_amd.ops import fp8

DEV = "cuda"


@pytest.mark.parametrize("N,per,limit", [(512, 6422528, (1 << 31) - 64),
                                         (7, 100, 250), (5, 10, 1000),
                                         (3, 400, 250)])
def test_image_chunks_cover_the_batch(monkeypatch, N, per, limit):
    monkeypatch.setattr(ops, "_BUF_MAX", limit)
    t = torch.empty(N, per, dtype=torch.uint8, device="meta")
    ch = ops._image_chunks(N, t, None)
    assert ch[0][0] == 0 and ch[-1][1] == N
    assert all(a[1] == b[0] for a, b in zip(ch, ch[1:]))
    sizes = [b - a for a, b in ch]
    assert max(sizes) - min(sizes) <= max(sizes) // 2 + 1
    if N * per < limit:
        assert ch == [(0, N)]
    elif per < limit:
        assert all(s * per < limit for s in sizes)
    else:
        assert sizes == [1] * N     # one image per launch is the floor


def _rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale)


def _three_chunks(monkeypatch, t):
    """make ``t`` (leading dim = images) split into three launches"""
    per = t.numel() // t.shape[0] * t.element_size()
    monkeypatch.setattr(ops, "_BUF_MAX", per * -(-t.shape[0] // 3) + 1)
    assert len(ops._image_chunks(t.shape[0], t)) == 3


CONVS = [
    # N, H, W, C, OC, K, pad, groups
    (7, 14, 14, 64, 64, 3, 1, 1),      # halo forward
    (7, 13, 13, 64, 128, 3, 1, 1),     # implicit GEMM (13 x 13: no halo)
    (6, 27, 27, 96, 256, 5, 2, 2),     # grouped
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONVS)
def test_chunked_conv_fwd_dgrad_bit_identical(monkeypatch, cfg):
    N, H, W, C, OC, K, p, g = cfg
    pad = (p, p, p, p)
    x = _rnd(N, H, W, C).to(DEV, torch.bfloat16)
    w = _rnd(OC, K, K, C // g, scale=0.05, seed=1).to(DEV, torch.bfloat16)
    b = _rnd(OC, seed=2).to(DEV)
    dy = _rnd(N, H, W, OC, scale=0.1, seed=3).to(DEV, torch.bfloat16)
    aux = _rnd(N, H, W, C, seed=4).to(DEV, torch.bfloat16)
    y0 = ops.conv_fwd(x, w, b, (1, 1), pad, g, 3)
    d0 = ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), pad, g, aux=aux,
                        aux_act=3)
    gw0 = torch.zeros(OC, K, K, C // g, device=DEV)
    gb0 = torch.zeros(OC, device=DEV)
    ops.conv_wgrad(x, dy, gw0, (1, 1), pad, g, dbias=gb0)
    _three_chunks(monkeypatch, x)
    y1 = ops.conv_fwd(x, w, b, (1, 1), pad, g, 3)
    monkeypatch.undo()
    _three_chunks(monkeypatch, dy)
    d1 = ops.conv_dgrad(dy, w, (N, H, W, C), (1, 1), pad, g, aux=aux,
                        aux_act=3)
    gw1 = torch.zeros(OC, K, K, C // g, device=DEV)
    gb1 = torch.zeros(OC, device=DEV)
    ops.conv_wgrad(x, dy, gw1, (1, 1), pad, g, dbias=gb1)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(d0, d1)
    tol = 1e-4 * gw0.abs().max().item()
    assert (gw0 - gw1).abs().max().item() <= tol
    assert (gb0 - gb1).abs().max().item() <= 1e-4 * gb0.abs().max().item()


@pytest.mark.gpu
def test_chunked_conv_fwd_q8_epilogue(monkeypatch):
    """the fused fp8 copy of a chunked forward lands at each chunk's
    offset"""
    N, H, W, C, OC = 7, 14, 14, 64, 64
    x = _rnd(N, H, W, C).to(DEV, torch.bfloat16)
    w = _rnd(OC, 3, 3, C, scale=0.05, seed=1).to(DEV, torch.bfloat16)
    b = _rnd(OC, seed=2).to(DEV)
    outs = []
    for chunked in (False, True):
        nxt = fp8.Scaler(DEV, fp8.E4M3)
        nxt.prime(torch.full((16,), 3.0, device=DEV))
        q8 = torch.zeros(N, H, W, OC, dtype=torch.float8_e4m3fn, device=DEV)
        if chunked:
            _three_chunks(monkeypatch, x)
        y = ops.conv_fwd(x, w, b, (1, 1), (1, 1, 1, 1), 1, 3, q8=q8,
                         q8_scaler=nxt)
        torch.cuda.synchronize()
        outs.append((y.clone(), q8.view(torch.uint8).clone(),
                     nxt.shard.clone()))
        monkeypatch.undo()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2].max(), outs[1][2].max())


@pytest.mark.gpu
def test_chunked_fp8_convs(monkeypatch):
    N, H, W, C, OC = 7, 14, 14, 64, 128
    sx, sw, sd = (fp8.Scaler(DEV, fp8.E4M3), fp8.Scaler(DEV, fp8.E4M3),
                  fp8.Scaler(DEV, fp8.E5M2))
    x8 = fp8.quantize(_rnd(N, H, W, C).to(DEV), sx)
    w8 = fp8.quantize(_rnd(OC, 3, 3, C, scale=0.05, seed=1).to(DEV), sw)
    d8 = fp8.quantize(_rnd(N, H, W, OC, scale=0.1, seed=3).to(DEV), sd)
    aux = _rnd(N, H, W, C, seed=4).to(DEV, torch.bfloat16)
    pad = (1, 1, 1, 1)
    res = []
    for chunked in (False, True):
        if chunked:
            _three_chunks(monkeypatch, x8)
        y = fp8.conv_fwd(x8, sx, w8, sw, None, (1, 1), pad, 1, 3)
        dx = fp8.conv_dgrad(d8, sd, w8, sw, (N, H, W, C), (1, 1), pad, 1,
                            aux=aux, aux_act=3)
        gw = torch.zeros(OC, 3, 3, C, device=DEV)
        fp8.conv_wgrad(x8, sx, d8, sd, gw, (1, 1), pad, 1)
        torch.cuda.synchronize()
        res.append((y, dx, gw))
        monkeypatch.undo()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    gw0, gw1 = res[0][2], res[1][2]
    assert (gw0 - gw1).abs().max().item() <= 1e-4 * gw0.abs().max().item()
