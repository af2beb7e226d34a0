"""FP8 path (veles_amd/ops/fp8.py, csrc/kernels/gemm_fp8.hip): delayed
scaling semantics and a float8 training run on the CPU reference; on the
MI355X every fp8 kernel against the CPU reference fed with the SAME
quantized operands (so only accumulation order differs), plus quantizer
bit-exactness against PyTorch's float8 casts."""
import numpy
import pytest
import torch

from veles_amd import ops
from veles_amd.ops import fp8
from veles_amd.utils.config import root

DEV = "cuda"


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed + sum(shape))
    return torch.randn(*shape, generator=g) * scale


def close(got, ref, tol):
    got, ref = got.float().cpu(), ref.float().cpu()
    err = (got - ref).abs().max().item()
    mag = ref.abs().max().item() + 1e-6
    assert err <= tol * mag, "max err %g vs scale %g (tol %g)" % (err, mag, tol)


# ------------------------------------------------------------------ CPU
def test_scaler_prime_record_roll_cpu():
    s = fp8.Scaler("cpu", fp8.E4M3)
    x = rnd(64, 32, scale=3.0)
    q = fp8.quantize(x, s)
    assert q.dtype == torch.float8_e4m3fn
    amax = x.abs().max().item()
    # primed from the tensor itself: amax maps to the format maximum
    assert abs(s.scale() - 448.0 / amax) < 1e-3 * s.scale()
    close(fp8.dequantize(q, s), x, 0.07)
    # the quantizer records this step's amax; roll moves it into history
    y = x * 4
    fp8.quantize(y, s)
    assert abs(s.state[fp8.HIST].item() - 4 * amax) < 1e-4 * amax
    s.registry.roll()
    assert s.state[fp8.HIST].item() == 0
    assert abs(s.scale() - 448.0 / (4 * amax)) < 1e-3 * s.scale()


def test_quantize_saturates_cpu():
    s = fp8.Scaler("cpu", fp8.E5M2)
    s.prime(torch.ones(4))           # scale = 57344
    q = fp8.quantize(torch.tensor([10.0, -10.0, 0.5]), s, record=False)
    assert torch.isfinite(q.float()).all()
    assert q.float()[0].item() == 57344.0 and q.float()[1].item() == -57344.0


def test_fp8_layer_policy_cpu(monkeypatch):
    """The 224-wide 64-channel convs stay on bf16 in an fp8 model (the bf16
    kernels beat the fp8 loops there, profiles/r6/vgg16_fp8_policy_ab_r6x.txt);
    every other eligible shape, and all of them under the override, run fp8."""
    monkeypatch.delenv("VELES_AMD_FP8_ALL_CONVS", raising=False)
    assert not fp8.fp8_conv_pays(64, 224, 224)      # VGG conv1_2
    assert fp8.fp8_conv_pays(64, 112, 112)          # VGG conv2_1
    assert fp8.fp8_conv_pays(128, 224, 224)
    assert fp8.fp8_conv_pays(512, 14, 14)
    monkeypatch.setenv("VELES_AMD_FP8_ALL_CONVS", "1")
    assert fp8.fp8_conv_pays(64, 224, 224)
    monkeypatch.delenv("VELES_AMD_FP8_ALL_CONVS")
    from veles_amd.utils.config import get
    old = get(root.common.engine.fp8_all_convs, False)
    root.common.engine.fp8_all_convs = True
    try:
        assert fp8.fp8_conv_pays(64, 224, 224)
    finally:
        root.common.engine.fp8_all_convs = old


def test_fp8_gemm_close_to_fp32_cpu():
    a, b = rnd(96, 256), rnd(80, 256, seed=1)
    sa, sb = fp8.Scaler("cpu"), fp8.Scaler("cpu")
    got = fp8.gemm(fp8.quantize(a, sa), sa, fp8.quantize(b, sb), sb)
    close(got, a @ b.t(), 0.06)


def test_float8_workflow_trains_cpu():
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    import veles_amd.loader  # noqa: F401
    g = {"learning_rate": 0.05, "gradient_moment": 0.9}
    layers = [
        {"type": "conv_str", "->": {"n_kernels": 16, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "all2all_str", "->": {"output_sample_shape": 64},
         "<-": dict(g)},
        {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": dict(g)}]
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "float8"
    try:
        torch.manual_seed(0)
        wf = StandardWorkflow(
            DummyLauncher(), loader_name="synthetic_images",
            loader_config={"dataset": "mnist", "class_lengths": (0, 100, 400),
                           "minibatch_size": 50, "normalization_type":
                           "mean_disp", "seed": 7, "noise": 110.0},
            layers=layers, decision_config={"max_epochs": 3,
                                            "fail_iterations": 100})
        wf.initialize(device=Device(backend="cpu"))
        f = wf.forwards
        assert not f[0].fp8_          # C = 1: bf16 / fp32 path
        assert f[1].fp8_ and f[3].fp8_ and not f[4].fp8_
        step0 = f[1].fp8_sx_.registry.step
        wf.run()
        h = wf.decision.history
        assert h[-1]["validation_loss"] < h[0]["validation_loss"]
        assert f[1].fp8_sx_.registry.step - step0 == wf.param_store_.steps
    finally:
        root.common.engine.precision_type = old


def _fp8_two_conv_run(fuse, steps=4, backend="cpu"):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    g = {"learning_rate": 0.05, "gradient_moment": 0.9}
    layers = [
        {"type": "conv_str", "->": {"n_kernels": 16, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": dict(g)}]
    old = (root.common.engine.precision_type,
           root.common.engine.fp8_fuse_quant)
    root.common.engine.precision_type = "float8"
    root.common.engine.fp8_fuse_quant = fuse
    try:
        random_generator.get().seed(5)
        numpy.random.seed(5)
        torch.manual_seed(0)
        wf = StandardWorkflow(
            DummyLauncher(), loader_name="synthetic_images",
            loader_config={"dataset": "mnist", "class_lengths": (0, 0, 400),
                           "minibatch_size": 50, "normalization_type":
                           "mean_disp", "seed": 7, "noise": 110.0,
                           "generate_on_device": False},
            layers=layers, decision_config={"max_epochs": None,
                                            "fail_iterations": None})
        wf.initialize(device=Device(backend=backend))
        wf.run_steps(steps)
        if backend == "hip":
            torch.cuda.synchronize()
        return wf
    finally:
        (root.common.engine.precision_type,
         root.common.engine.fp8_fuse_quant) = old


def test_fused_fp8_quantisation_matches_separate_pass_cpu():
    """conv -> fp8 conv -> fp8 conv -> 2x2 pool -> fp8 conv: from step 1 on
    the producing conv's epilogue / the pooling kernel writes the next fp8
    conv's e4m3 input copy, and in the backward the GD / pooling-GD kernel
    the e5m2 gradient copy of the fp8 conv GD below it (no quantize pass for
    them); training is identical to the separate-pass run."""
    a = _fp8_two_conv_run(False)
    b = _fp8_two_conv_run(True)
    f = b.forwards
    assert f[1].fp8_ and f[2].fp8_ and f[4].fp8_
    assert f[1].fp8_input_consumer() is f[2]
    from veles_amd.models.conv import fp8_input_consumer
    from veles_amd.models.gd_conv import fp8_grad_consumer
    assert fp8_input_consumer(f[3]) is f[4]        # pool -> fp8 conv
    gd = {id(u.forward): u for u in b.gds}
    assert gd[id(f[2])].fp8_grad_consumer() is gd[id(f[1])]
    assert fp8_grad_consumer(gd[id(f[3])]) is gd[id(f[2])]  # pool GD
    assert torch.equal(a.param_store_.master, b.param_store_.master)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [fp8.E4M3, fp8.E5M2])
def test_quantize_matches_torch_cast(fmt):
    x = rnd(4099, scale=2.0)          # odd length: vector body + tail
    s_cpu, s_gpu = fp8.Scaler("cpu", fmt), fp8.Scaler(DEV, fmt)
    q_cpu = fp8.quantize(x, s_cpu)
    q_gpu = fp8.quantize(x.to(DEV).to(torch.bfloat16).float(), s_gpu)
    xb = x.to(torch.bfloat16).float()
    q_ref = fp8.quantize(xb, fp8.Scaler("cpu", fmt))
    torch.cuda.synchronize()
    assert abs(s_gpu.scale() - s_cpu.scale()) < 1e-2 * s_cpu.scale()
    diff = (q_gpu.cpu().view(torch.uint8) != q_ref.view(torch.uint8))
    assert diff.sum().item() == 0, "%d of %d codes differ" % (
        diff.sum().item(), x.numel())
    assert q_cpu.shape == q_gpu.shape
    # amax recorded on the device
    assert abs(s_gpu.state[fp8.HIST].item() - xb.abs().max().item()) < 1e-6


def _pair(x, fmt=fp8.E4M3):
    """Quantize on the GPU; return (gpu q, gpu scaler, cpu copy, cpu scaler
    with the same state) so the reference sees identical operands."""
    s = fp8.Scaler(DEV, fmt)
    q = fp8.quantize(x.to(DEV).to(torch.bfloat16), s)
    torch.cuda.synchronize()
    sc = fp8.Scaler("cpu", fmt)
    sc.state.copy_(s.state.cpu())
    sc.primed = True
    return q, s, q.cpu(), sc


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (300, 200, 512),
                                   (1000, 96, 784 + 16), (7, 9, 32)])
def test_gemm_fp8(M, N, K):
    a8, sa, a8c, sac = _pair(rnd(M, K))
    b8, sb, b8c, sbc = _pair(rnd(N, K, seed=1, scale=0.1))
    bias = torch.randn(N)
    aux = rnd(M, N, seed=3).to(torch.bfloat16)
    for act, auxt in ((0, None), (3, None), (0, aux)):
        ref = fp8.gemm(a8c, sac, b8c, sbc, bias=bias, act=act,
                       aux=auxt, aux_act=3)
        got = fp8.gemm(a8, sa, b8, sb, bias=bias.to(DEV), act=act,
                       aux=None if auxt is None else auxt.to(DEV), aux_act=3)
        torch.cuda.synchronize()
        close(got, ref, 1e-2)


@pytest.mark.gpu
def test_gemm_fp8_e5m2_a_operand():
    a8, sa, a8c, sac = _pair(rnd(256, 256, scale=1e-3), fp8.E5M2)
    b8, sb, b8c, sbc = _pair(rnd(192, 256, seed=2))
    got = fp8.gemm(a8, sa, b8, sb)
    ref = fp8.gemm(a8c, sac, b8c, sbc)
    close(got, ref, 1e-2)


CONVS8 = [
    # N, H, W, C, OC, KH, KW, sliding(x,y), padding(l,t,r,b), groups
    (2, 14, 14, 64, 64, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (2, 13, 13, 32, 48, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (2, 27, 27, 96, 256, 5, 5, (1, 1), (2, 2, 2, 2), 2),
    (3, 11, 9, 16, 32, 3, 3, (2, 2), (1, 1, 0, 0), 1),
    (2, 8, 8, 128, 160, 1, 1, (1, 1), (0, 0, 0, 0), 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONVS8)
def test_conv_fwd_fp8(cfg):
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    x8, sx, x8c, sxc = _pair(rnd(N, H, W, C))
    w8, sw, w8c, swc = _pair(rnd(OC, KH, KW, C // g, seed=1, scale=0.1))
    b = torch.randn(OC)
    for act in (0, 3):
        ref = fp8.conv_fwd(x8c, sxc, w8c, swc, b, sl, pad, g, act)
        got = fp8.conv_fwd(x8, sx, w8, sw, b.to(DEV), sl, pad, g, act)
        torch.cuda.synchronize()
        close(got, ref, 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CONVS8)
def test_conv_dgrad_fp8(cfg):
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    OH, OW = ops.conv_out_size(H, W, KH, KW, sl, pad)
    d8, sd, d8c, sdc = _pair(rnd(N, OH, OW, OC, seed=2, scale=1e-2),
                             fp8.E5M2)
    w8, sw, w8c, swc = _pair(rnd(OC, KH, KW, C // g, seed=1, scale=0.1))
    aux = rnd(N, H, W, C, seed=3).to(torch.bfloat16)
    ref = fp8.conv_dgrad(d8c, sdc, w8c, swc, (N, H, W, C), sl, pad, g,
                         aux=aux, aux_act=3)
    got = fp8.conv_dgrad(d8, sd, w8, sw, (N, H, W, C), sl, pad, g,
                         aux=aux.to(DEV), aux_act=3)
    torch.cuda.synchronize()
    close(got, ref, 1e-2)


WGRAD8 = CONVS8 + [
    # several K tiles / splits, OC and KK off the 128 grid, 7 x 7 images
    (4, 28, 28, 64, 128, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (8, 14, 14, 256, 160, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (16, 7, 7, 48, 32, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    # the fp8 halo kernel (wgrad_halo.hip): full-row windows with steps
    # across images (13 / 56-wide), segment windows (112 / 224-wide)
    (3, 13, 13, 256, 384, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (2, 56, 56, 64, 128, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (1, 112, 112, 64, 128, 3, 3, (1, 1), (1, 1, 1, 1), 1),
    (1, 224, 224, 64, 64, 3, 3, (1, 1), (1, 1, 1, 1), 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", WGRAD8)
def test_conv_wgrad_fp8(cfg):
    """e5m2 gradient x e4m3 input weight gradient (wgrad_fp8.hip, transposed
    LDS reads) against the float32 weight gradient of the same dequantized
    operands; accumulates into the gradient, any pixel split"""
    N, H, W, C, OC, KH, KW, sl, pad, g = cfg
    OH, OW = ops.conv_out_size(H, W, KH, KW, sl, pad)
    x8, sx, x8c, sxc = _pair(rnd(N, H, W, C))
    d8, sd, d8c, sdc = _pair(rnd(N, OH, OW, OC, seed=2, scale=1e-2),
                             fp8.E5M2)
    ref = torch.zeros(OC, KH, KW, C // g)
    refb = torch.zeros(OC)
    fp8.conv_wgrad(x8c, sxc, d8c, sdc, ref, sl, pad, g, dbias=refb)
    for splits in (1, 3, None):
        got = torch.ones(OC, KH, KW, C // g, device=DEV)
        gotb = torch.ones(OC, device=DEV)
        fp8.conv_wgrad(x8, sx, d8, sd, got, sl, pad, g, splits=splits,
                       dbias=gotb)
        torch.cuda.synchronize()
        close(got - 1.0, ref, 2e-3)
        close(gotb - 1.0, refb, 2e-3)


@pytest.mark.gpu
def test_fp8_workflow_wgrad_fp8_vs_bf16():
    """the same fp8 conv stack trained a few steps with the weight
    gradients on the fp8 kernel and on the bf16 kernel: the fp8 wgrad path
    is taken, and the trajectories agree to the fp8 gradient rounding"""
    old = root.common.engine.fp8_wgrad
    try:
        root.common.engine.fp8_wgrad = False
        a = _fp8_two_conv_run(True, steps=3, backend="hip")
        root.common.engine.fp8_wgrad = True
        b = _fp8_two_conv_run(True, steps=3, backend="hip")
    finally:
        root.common.engine.fp8_wgrad = old
    gd = [u for u in b.gds if getattr(u.forward, "fp8_", False)]
    assert gd and all(u._fp8_wgrad_ok(u.forward, u.forward.x8_) for u in gd)
    w0 = _fp8_two_conv_run(True, steps=0, backend="hip").param_store_ \
        .master.float().cpu()
    da = a.param_store_.master.float().cpu() - w0
    db = b.param_store_.master.float().cpu() - w0
    assert torch.isfinite(db).all() and db.norm() > 0
    rel = ((da - db).norm() / da.norm()).item()
    assert 0 < rel < 0.3, rel


@pytest.mark.gpu
def test_fp8_roll_kernel():
    r = fp8.registry(DEV)
    s = fp8.Scaler(DEV)
    s.prime(torch.full((64,), 2.0, device=DEV))
    fp8.quantize(torch.full((64,), 8.0, device=DEV), s)
    step = r.step
    r.roll()
    torch.cuda.synchronize()
    st = s.state.cpu()
    assert st[fp8.HIST].item() == 0
    assert st[step % fp8.HIST].item() == 8.0
    assert abs(s.scale() - 448.0 / 8.0) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("dgrad", [False, True])
def test_fused_quantisation_epilogue(dgrad):
    """The fp8 conv epilogue's fused copy for the next layer equals a
    separate quantize pass of the bf16 output at the consumer scaler's
    scale, and its amax reaches the history at the roll."""
    N, H, W, C, OC = 4, 14, 14, 32, 48
    nxt = fp8.Scaler(DEV, fp8.E5M2 if dgrad else fp8.E4M3)
    nxt.prime(torch.full((16,), 3.0, device=DEV))
    w8, sw, _, _ = _pair(rnd(OC, 3, 3, C, seed=1, scale=0.1))
    if not dgrad:
        x8, sx, _, _ = _pair(rnd(N, H, W, C))
        q8 = torch.empty(N, H, W, OC, dtype=fp8.TORCH_DT[nxt.fmt],
                         device=DEV)
        y = fp8.conv_fwd(x8, sx, w8, sw, None, (1, 1), (1, 1, 1, 1), 1, 3,
                         q8=q8, q8_scaler=nxt)
    else:
        d8, sd, _, _ = _pair(rnd(N, H, W, OC, seed=2, scale=1e-2), fp8.E5M2)
        q8 = torch.empty(N, H, W, C, dtype=fp8.TORCH_DT[nxt.fmt], device=DEV)
        aux = rnd(N, H, W, C, seed=3).to(torch.bfloat16).to(DEV)
        y = fp8.conv_dgrad(d8, sd, w8, sw, (N, H, W, C), (1, 1),
                           (1, 1, 1, 1), 1, aux=aux, aux_act=3, q8=q8,
                           q8_scaler=nxt)
    torch.cuda.synchronize()
    ref = fp8.quantize(y, nxt, record=False)
    torch.cuda.synchronize()
    assert torch.equal(q8.view(torch.uint8), ref.view(torch.uint8))
    r = nxt.registry
    step = r.step
    r.roll()
    torch.cuda.synchronize()
    amax = y.float().abs().max().item()
    assert nxt.state[step % fp8.HIST].item() == amax
    assert nxt.shard.abs().max().item() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    # VGG conv1_1 (C = 3 -> channel-padded, halo kernel), a strided conv
    # (implicit GEMM), a grouped conv with 24 outputs per group
    (2, 24, 24, 3, 64, 3, (1, 1), 1, 1),
    (2, 17, 17, 32, 48, 3, (2, 2), 1, 1),
    (2, 12, 12, 48, 48, 3, (1, 1), 1, 2)])
def test_fused_quantisation_bf16_conv(cfg):
    """A bf16 conv feeding an fp8 conv writes that conv's e4m3 input copy
    from its epilogue: equal to a separate quantize pass of its bf16
    output, amax in the shards; the bf16 output is unchanged"""
    N, H, W, C, OC, k, sl, p, g = cfg
    x = rnd(N, H, W, C).to(torch.bfloat16).to(DEV)
    w = rnd(OC, k, k, C // g, seed=1, scale=0.1).to(torch.bfloat16).to(DEV)
    b = torch.randn(OC, device=DEV)
    nxt = fp8.Scaler(DEV, fp8.E4M3)
    nxt.prime(torch.full((16,), 3.0, device=DEV))
    pad = (p, p, p, p)
    plain = ops.conv_fwd(x, w, b, sl, pad, g, 3)
    OH, OW = ops.conv_out_size(H, W, k, k, sl, pad)
    q8 = torch.empty(N, OH, OW, OC, dtype=fp8.TORCH_DT[nxt.fmt], device=DEV)
    y = ops.conv_fwd(x, w, b, sl, pad, g, 3, q8=q8, q8_scaler=nxt)
    torch.cuda.synchronize()
    assert torch.equal(y, plain)
    ref = fp8.quantize(y, nxt, record=False)
    torch.cuda.synchronize()
    assert torch.equal(q8.view(torch.uint8), ref.view(torch.uint8))
    r = nxt.registry
    step = r.step
    r.roll()
    torch.cuda.synchronize()
    assert nxt.state[step % fp8.HIST].item() == y.float().abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("bwd", [False, True])
@pytest.mark.parametrize("chunked", [False, True])
def test_fused_quantisation_pool2(bwd, chunked, monkeypatch):
    """The 2 x 2 pooling kernels' fused fp8 copy of their result equals a
    separate quantize pass at the consumer scaler's scale; the amax reaches
    the history at the roll.  ``chunked``: one launch per image (the path
    past 2^31 elements, threshold lowered), the amax of all of them."""
    N, H, W, C = 3, 16, 14, 32
    if chunked:
        monkeypatch.setattr(ops, "_CHUNK_ELEMS", H * W * C + 1)
    nxt = fp8.Scaler(DEV, fp8.E5M2 if bwd else fp8.E4M3)
    nxt.prime(torch.full((16,), 2.0, device=DEV))
    x = rnd(N, H, W, C).to(torch.bfloat16).to(DEV)
    if not bwd:
        q8 = torch.empty(N, H // 2, W // 2, C, dtype=fp8.TORCH_DT[nxt.fmt],
                         device=DEV)
        y = ops.pool2_fwd(x, "max", q8=q8, q8_scaler=nxt)
    else:
        dy = rnd(N, H // 2, W // 2, C, seed=4).to(torch.bfloat16).to(DEV)
        q8 = torch.empty(N, H, W, C, dtype=fp8.TORCH_DT[nxt.fmt], device=DEV)
        y = ops.pool2_bwd(x, dy, "max", aux=x, aux_act=3, q8=q8,
                          q8_scaler=nxt)
    torch.cuda.synchronize()
    ref = fp8.quantize(y, nxt, record=False)
    torch.cuda.synchronize()
    assert torch.equal(q8.view(torch.uint8), ref.view(torch.uint8))
    r = nxt.registry
    step = r.step
    r.roll()
    torch.cuda.synchronize()
    assert nxt.state[step % fp8.HIST].item() == y.float().abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 1024), (4100, 4000, 384),
                                   (8192, 2304, 128), (4096, 4096, 256 + 16)])
def test_gemm_fp8_pingpong_256(M, N, K):
    """The 256 x 256 fp8 ping-pong loop (gemm_pp256_fp8_kernel; >= 256 tiles)
    against the 128-row fp8 loop (hvk_set_fp8_variant(70)): the same MFMAs
    over the same K order, so bit-identical - and both against the float32
    product of the dequantised operands.  Covers partial row / column tiles,
    a one-tile K (prologue only) and a K tail."""
    a8, sa, a8c, sac = _pair(rnd(M, K))
    b8, sb, b8c, sbc = _pair(rnd(N, K, seed=1, scale=0.1))
    bias = torch.randn(N, device=DEV)
    lib = ops._lib.lib()
    outs = []
    try:
        for v in (70, -1):
            lib.hvk_set_fp8_variant(v)
            outs.append(fp8.gemm(a8, sa, b8, sb, bias=bias, act=3).clone())
    finally:
        lib.hvk_set_fp8_variant(-1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = torch.relu(fp8.dequantize(a8, sa).float() @
                     fp8.dequantize(b8, sb).float().t() + bias)
    close(outs[1], ref, 1e-2)


T4CONVS8 = [
    # N, H, W, C, OC, k, pad, groups, stride: VGG-like (128 / 256 / 512 outputs),
    # the AlexNet conv2 grouping, a stride-2 forward, partial row tiles
    (2, 28, 28, 64, 128, 3, 1, 1, 1),
    (3, 14, 14, 128, 256, 3, 1, 1, 1),
    (1, 7, 7, 256, 512, 3, 1, 1, 1),
    (2, 27, 27, 96, 256, 5, 2, 2, 1),
    (2, 16, 16, 64, 128, 3, 1, 1, 2),   # stride 2: forward only
    # 64 outputs per group: the 256 x 64 tiles (VGG conv1_2), partial tiles,
    # grouped
    (2, 30, 30, 64, 64, 3, 1, 1, 1),
    (2, 14, 14, 128, 128, 3, 1, 2, 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", T4CONVS8)
def test_conv_fp8_t4_loop(cfg):
    """The 192 x 128 (and 256 x 64) two-workgroups-per-CU fp8 loop
    (gemm_t4_fp8_kernel) against the 128-row fp8 loop
    (hvk_set_fp8_variant(71)): forward and
    backward-data bit-identical (same MFMAs, same K order), and against the
    float32 reference."""
    N, H, W, C, OC, k, p, g, s = cfg
    pad = (p, p, p, p)
    x8, sx, x8c, sxc = _pair(rnd(N, H, W, C))
    w8, sw, w8c, swc = _pair(rnd(OC, k, k, C // g, seed=1, scale=0.1))
    b = torch.randn(OC)
    lib = ops._lib.lib()
    try:
        outs = []
        # 71: 128-row loop; T4 with -1: the f32-staged epilogue, 73: the
        # register epilogue (bf16 C image), 74: the direct epilogue
        for v in (71, -1, 73, 74):
            lib.hvk_set_fp8_variant(v)
            outs.append(fp8.conv_fwd(x8, sx, w8, sw, b.to(DEV), (s, s), pad,
                                     g, 3).clone())
        for o in outs[1:]:
            assert torch.equal(outs[0], o)
        close(outs[1], fp8.conv_fwd(x8c, sxc, w8c, swc, b, (s, s), pad, g, 3),
              1e-2)
        # the fused e4m3 copy for the next layer: direct and staged epilogue
        # write the same bytes and the same amax
        q8s = []
        for v in (-1, 73, 74):
            lib.hvk_set_fp8_variant(v)
            nxt = fp8.Scaler(DEV, fp8.E4M3)
            nxt.prime(torch.full((16,), 3.0, device=DEV))
            q8 = torch.zeros(outs[0].shape, dtype=torch.float8_e4m3fn,
                             device=DEV)
            fp8.conv_fwd(x8, sx, w8, sw, b.to(DEV), (s, s), pad, g, 3,
                         q8=q8, q8_scaler=nxt)
            torch.cuda.synchronize()
            q8s.append((q8.view(torch.uint8).clone(), nxt.shard.max().item()))
        for q in q8s[1:]:
            assert torch.equal(q8s[0][0], q[0])
            assert q8s[0][1] == q[1] > 0
        if s == 1:
            OH, OW = ops.conv_out_size(H, W, k, k, (1, 1), pad)
            d8, sd, d8c, sdc = _pair(rnd(N, OH, OW, OC, seed=2, scale=1e-2),
                                     fp8.E5M2)
            outs = []
            for v in (71, -1, 73, 74):
                lib.hvk_set_fp8_variant(v)
                outs.append(fp8.conv_dgrad(d8, sd, w8, sw, (N, H, W, C),
                                           (1, 1), pad, g).clone())
            for o in outs[1:]:
                assert torch.equal(outs[0], o)
            close(outs[1], fp8.conv_dgrad(d8c, sdc, w8c, swc, (N, H, W, C),
                                          (1, 1), pad, g), 1e-2)
    finally:
        lib.hvk_set_fp8_variant(-1)


PP8CONVS = [
    # N, H, W, C, OC, k, pad, groups: >= 256 outputs (inputs, for the
    # backward-data) per group
    (3, 14, 14, 128, 256, 3, 1, 1),     # forward only: C = 128
    (1, 7, 7, 256, 512, 3, 1, 1),
    (2, 7, 7, 512, 512, 3, 1, 2),
    (2, 13, 13, 384, 256, 3, 1, 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", PP8CONVS)
def test_conv_fp8_pp256_loop(cfg):
    """fp8 convolutions on the 256 x 256 ping-pong loop (forced by
    hvk_set_fp8_variant(75)) against the 128-row fp8 loop (71): forward and
    backward-data bit-identical, the fused e4m3 copy too, and against the
    float32 reference"""
    N, H, W, C, OC, k, p, g = cfg
    pad = (p, p, p, p)
    x8, sx, x8c, sxc = _pair(rnd(N, H, W, C))
    w8, sw, w8c, swc = _pair(rnd(OC, k, k, C // g, seed=1, scale=0.1))
    b = torch.randn(OC)
    lib = ops._lib.lib()
    try:
        outs = []
        for v in (71, 75):
            lib.hvk_set_fp8_variant(v)
            nxt = fp8.Scaler(DEV, fp8.E4M3)
            nxt.prime(torch.full((16,), 3.0, device=DEV))
            q8 = torch.zeros(N, H, W, OC, dtype=torch.float8_e4m3fn,
                             device=DEV)
            y = fp8.conv_fwd(x8, sx, w8, sw, b.to(DEV), (1, 1), pad, g, 3,
                             q8=q8, q8_scaler=nxt)
            torch.cuda.synchronize()
            outs.append((y.clone(), q8.view(torch.uint8).clone(),
                         nxt.shard.max().item()))
        assert torch.equal(outs[0][0], outs[1][0])
        assert torch.equal(outs[0][1], outs[1][1])
        assert outs[0][2] == outs[1][2]
        close(outs[1][0], fp8.conv_fwd(x8c, sxc, w8c, swc, b, (1, 1), pad, g,
                                       3), 1e-2)
        if C // g >= 256:
            d8, sd, d8c, sdc = _pair(rnd(N, H, W, OC, seed=2, scale=1e-2),
                                     fp8.E5M2)
            outs = []
            for v in (71, 75):
                lib.hvk_set_fp8_variant(v)
                outs.append(fp8.conv_dgrad(d8, sd, w8, sw, (N, H, W, C),
                                           (1, 1), pad, g).clone())
            assert torch.equal(outs[0], outs[1])
            close(outs[1], fp8.conv_dgrad(d8c, sdc, w8c, swc, (N, H, W, C),
                                          (1, 1), pad, g), 1e-2)
    finally:
        lib.hvk_set_fp8_variant(-1)


@pytest.mark.gpu
def test_fp8_fc_dgrad_transposed_weights():
    """The fp8 FC backward-data of models/gd.py: e5m2 err against the
    transposed e4m3 weight copy (same scaler) equals the float32 product of
    the dequantised operands, with the derivative of the layer below"""
    from veles_amd.models.gd import GradientDescent
    B, n_in, n_out = 256, 1024, 512
    err = (rnd(B, n_out, scale=1e-2)).to(DEV).to(torch.bfloat16)
    W = (rnd(n_out, n_in, seed=1, scale=0.05)).to(DEV).to(torch.bfloat16)
    aux = rnd(B, n_in, seed=3).to(DEV).to(torch.bfloat16)

    class _Fwd:
        fp8_ = True

    fwd = _Fwd()
    fwd.fp8_sw_ = fp8.Scaler(DEV, fp8.E4M3)
    fwd.w8_ = fp8.quantize(W, fwd.fp8_sw_)
    gd = GradientDescent.__new__(GradientDescent)
    gd.e8_ = gd.wt8_ = gd.fp8_se_ = None
    out = torch.empty(B, n_in, dtype=torch.bfloat16, device=DEV)
    gd._fp8_dgrad(fwd, err, out, aux, 3)
    torch.cuda.synchronize()
    ref = (fp8.dequantize(gd.e8_, gd.fp8_se_).float() @
           fp8.dequantize(fwd.w8_, fwd.fp8_sw_).float()) * \
        (aux.float() > 0).float()
    close(out, ref, 1e-2)
    assert torch.equal(gd.wt8_.view(torch.uint8).cpu(),
                       fwd.w8_.view(torch.uint8).t().cpu())


@pytest.mark.gpu
def test_conv_wgrad_fp8_halo_taken_and_matches_gemm_kernel():
    """VGG-like stride-1 shapes take the fp8 halo weight gradient; it equals
    the wgrad_fp8.hip kernel's result to f32 rounding (same fp8 operands,
    same scales)"""
    N, H, W, C, OC = 2, 56, 56, 128, 128
    x8, sx, _, _ = _pair(rnd(N, H, W, C))
    d8, sd, _, _ = _pair(rnd(N, H, W, OC, seed=2, scale=1e-2), fp8.E5M2)
    geo = (N, H, W, C, OC, 3, 3, 1, 1, H, W, 1, 0, sx.fmt, sd.fmt,
           sx.state.data_ptr(), sd.state.data_ptr(), fp8.HIST,
           float(sx.fmax_eff), float(sd.fmax_eff), 0)
    assert ops._lib.lib().hvk_conv_wgrad_halo_fp8(
        x8.data_ptr(), d8.data_ptr(), 0, 0, None, *geo) > 0
    res = {}
    try:
        for on in (True, False):
            ops.set_halo_wgrad(on)
            got = torch.zeros(OC, 3, 3, C, device=DEV)
            gotb = torch.zeros(OC, device=DEV)
            fp8.conv_wgrad(x8, sx, d8, sd, got, (1, 1), (1, 1, 1, 1), 1,
                           dbias=gotb)
            res[on] = (got, gotb)
    finally:
        ops.set_halo_wgrad(True)
    torch.cuda.synchronize()
    close(res[True][0], res[False][0], 1e-5)
    close(res[True][1], res[False][1], 1e-5)
