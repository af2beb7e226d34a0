"""Device tuning table (veles_amd/ops/autotune.py): JSON round trip, lookups
overriding the built-in split-K heuristics per shape, call recording, and on
the GPU a tuning pass whose choices keep the numerics."""
import json

import pytest
import torch

from veles_amd import ops
from veles_amd.ops import autotune


@pytest.fixture
def tab(tmp_path, monkeypatch):
    t = autotune.TuningTable(str(tmp_path / "gfx950.json"))
    monkeypatch.setattr(autotune, "_TABLE", t)
    monkeypatch.setattr(autotune, "_ENABLED", True)
    return t


def test_table_round_trip_and_bad_files(tmp_path):
    p = str(tmp_path / "t.json")
    t = autotune.TuningTable(p)
    assert t.entries == {} and t.get("wgrad:1:2:3:1") is None
    t.set(autotune.key("wgrad", 1, 2, 3, 1), 8, 10.5, 4, 12.0)
    t.data["device"] = {"name": "x"}
    t.save()
    u = autotune.TuningTable(p)
    assert u.get("wgrad:1:2:3:1") == 8
    assert u.entries["wgrad:1:2:3:1"]["default_us"] == 12.0
    assert u.data["device"]["name"] == "x"
    for bad in ("{not json", json.dumps({"format": 99, "entries": {}}),
                json.dumps([1, 2])):
        with open(p, "w") as f:
            f.write(bad)
        v = autotune.TuningTable(p)
        assert v.entries == {}   # ignored, built-in defaults apply


def test_wgrad_split_lookup_and_recording(tab):
    x = torch.zeros(2, 9, 9, 16)
    dy = torch.zeros(2, 7, 7, 32)
    dw = torch.zeros(32, 3, 3, 16)
    shape = (2 * 7 * 7, 32, 3 * 3 * 16 + 1, 1)
    default = ops.wgrad_splits(*shape)
    autotune.record(True)
    try:
        assert ops._wgrad_splits_for(x, dy, dw, (1, 1), (0, 0, 0, 0), 1,
                                     shape) == default
        tab.set(autotune.key("wgrad", *shape), default + 3)
        assert ops._wgrad_splits_for(x, dy, dw, (1, 1), (0, 0, 0, 0), 1,
                                     shape) == default + 3
        log = autotune.recorded()
    finally:
        autotune.record(False)
    kind, g = log[autotune.key("wgrad", *shape)]
    assert kind == "wgrad" and g["x"] == (2, 9, 9, 16)
    assert g["default"] == default and g["groups"] == 1


def test_splitk_lookup(tab, monkeypatch):
    M, N, K = 256, 512, 4096
    a = torch.zeros(M, K)
    b = torch.zeros(N, K)
    out = torch.zeros(M, N)
    default = ops.auto_splitk(M, N, K, out)
    assert default > 1
    assert ops._splitk_for(a, b, False, True, out, M, N, K, None,
                           None) == default
    tab.set(autotune.key("splitk", M, N, K), 0)
    assert ops._splitk_for(a, b, False, True, out, M, N, K, None, None) == 0
    tab.set(autotune.key("splitk", M, N, K), 6)
    assert ops._splitk_for(a, b, False, True, out, M, N, K, None, None) == 6
    # misaligned rows: never split, whatever the table says
    out2 = torch.zeros(M, N + 4)[:, :N]
    assert ops._splitk_for(a, b, False, True, out2, M, N, K, None,
                           None) == 0 or out2.stride(0) % 8 == 0
    monkeypatch.setattr(autotune, "_ENABLED", False)
    assert ops._splitk_for(a, b, False, True, out, M, N, K, None,
                           None) == default


@pytest.mark.gpu
def test_tune_keeps_numerics(tab):
    """Record one conv weight gradient and one split-K FC GEMM, tune them,
    and check the tuned choices give the default's results."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(8, 30, 30, 64, device=dev, generator=g).bfloat16()
    dy = torch.randn(8, 28, 28, 96, device=dev, generator=g).bfloat16()
    a = torch.randn(256, 4096, device=dev, generator=g).bfloat16()
    w = torch.randn(1024, 4096, device=dev, generator=g).bfloat16()

    def run():
        dw = torch.zeros(96, 3, 3, 64, device=dev)
        ops.conv_wgrad(x, dy, dw)
        y = ops.gemm(a, w, trans_b=True)
        torch.cuda.synchronize()
        return dw, y

    autotune.record(True)
    try:
        dw0, y0 = run()
        log = autotune.recorded()
    finally:
        autotune.record(False)
    assert {k.split(":")[0] for k in log} == {"wgrad", "splitk"}
    autotune.tune(log, repeats=2, tab=tab, verbose=False)
    assert set(tab.entries) == set(log)
    for e in tab.entries.values():
        assert e["us"] > 0 and e["us"] <= e["default_us"]
    dw1, y1 = run()
    torch.testing.assert_close(dw1, dw0, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(y1.float(), y0.float(), rtol=2e-2, atol=2e-2)
    ref = (a.float() @ w.float().t())
    torch.testing.assert_close(y1.float(), ref, rtol=2e-2, atol=0.5)


def test_wgrad_geometry_checked_and_logical_shape_logged(tab):
    """A weight gradient whose x / dy / dw disagree raises on the host (the
    kernels would read out of bounds); a call logged with a shape tuple (the
    s2d path logs the logical image, not the s2d data) keeps it."""
    x = torch.zeros(2, 9, 9, 16)
    dw = torch.zeros(32, 3, 3, 16)
    with pytest.raises(ValueError):   # dy 6x6, geometry says 7x7
        ops.conv_wgrad(x, torch.zeros(2, 6, 6, 32), dw)
    with pytest.raises(ValueError):   # dw for 3 input channels
        ops.conv_wgrad(x, torch.zeros(2, 7, 7, 32), torch.zeros(32, 3, 3, 3))
    shape = (2 * 7 * 7, 32, 3 * 3 * 16 + 1, 1)
    autotune.record(True)
    try:
        ops._wgrad_splits_for((2, 9, 9, 16), torch.zeros(2, 7, 7, 32), dw,
                              (1, 1), (0, 0, 0, 0), 1, shape)
        log = autotune.recorded()
    finally:
        autotune.record(False)
    assert log[autotune.key("wgrad", *shape)][1]["x"] == (2, 9, 9, 16)


@pytest.mark.gpu
def test_tune_replays_s2d_weight_gradient(tab):
    """AlexNet conv1's weight gradient takes the loader's space-to-depth image
    (ops.S2DImage).  The autotuner must replay it on a plain image of the
    logical shape (it once replayed the s2d data as the image and faulted)."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(4, 227, 227, 3, device=dev, generator=g).bfloat16()
    pad = (0, 0, 0, 0)
    OH, OW = ops.conv_out_size(227, 227, 11, 11, (4, 4), pad)
    dy = torch.randn(4, OH, OW, 96, device=dev, generator=g).bfloat16()
    s2 = ops.S2DImage(ops.space_to_depth(x, 4, 11, 11, pad), 4, x.shape)

    def run(inp):
        dw = torch.zeros(96, 11, 11, 3, device=dev)
        ops.conv_wgrad(inp, dy, dw, (4, 4), pad)
        torch.cuda.synchronize()
        return dw

    # the split-K GEMM path the tuner records (the halo weight gradient,
    # the default for this shape, sizes its own pixel split)
    halo = ops._HALO_WGRAD
    ops.set_halo_wgrad(False)
    try:
        autotune.record(True)
        try:
            dw0 = run(s2)
            log = autotune.recorded()
        finally:
            autotune.record(False)
        (k, (kind, gm)), = log.items()
        assert kind == "wgrad" and gm["x"] == (4, 227, 227, 3)
        autotune.tune(log, repeats=2, tab=tab, verbose=False)
        torch.testing.assert_close(run(x), dw0, rtol=1e-4, atol=1e-2)
    finally:
        ops.set_halo_wgrad(halo)
    ref = torch.nn.grad.conv2d_weight(
        x.permute(0, 3, 1, 2).float(), (96, 3, 11, 11),
        dy.permute(0, 3, 1, 2).float(), stride=4).permute(0, 2, 3, 1)
    torch.testing.assert_close(dw0, ref, rtol=2e-2, atol=0.5)


def test_conv_fwd_dgrad_geometry_checked():
    x = torch.zeros(2, 9, 9, 16)
    w = torch.zeros(32, 3, 3, 16)
    with pytest.raises(ValueError):
        ops.conv_fwd(x, w, out=torch.zeros(2, 6, 6, 32))
    with pytest.raises(ValueError):   # dy 6x6 for a 9x9 input, 3x3 kernel
        ops.conv_dgrad(torch.zeros(2, 6, 6, 32), w, (2, 9, 9, 16))
    with pytest.raises(ValueError):   # aux of the wrong shape
        ops.conv_dgrad(torch.zeros(2, 7, 7, 32), w, (2, 9, 9, 16),
                       aux=torch.zeros(2, 8, 8, 16), aux_act=1)
    assert ops.conv_dgrad(torch.zeros(2, 7, 7, 32), w,
                          (2, 9, 9, 16)).shape == (2, 9, 9, 16)
