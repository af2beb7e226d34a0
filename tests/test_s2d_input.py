"""The loader gather fused with the first conv's space-to-depth transform
(ops.fill_minibatch_s2d / hvk_fill_minibatch_s2d, FullBatchLoader
.request_s2d_input): the s2d image it writes equals space_to_depth of the
normalised image, and a conv on it equals the strided conv on the image."""
import numpy
import pytest
import torch
import torch.nn.functional as F

from veles_amd import ops

GEOM = [(4, 11, 11, (0, 0, 0, 0), 227, 227),     # AlexNet conv1
        (4, 11, 11, (2, 2, 2, 2), 61, 53),
        (4, 8, 8, (1, 3, 1, 3), 40, 37)]


def _data(n=13, H=227, W=227, seed=0):
    g = numpy.random.default_rng(seed)
    src = torch.from_numpy(g.integers(0, 256, (n, H, W, 3), dtype=numpy.uint8))
    mean = torch.from_numpy(g.uniform(60, 180, H * W * 3).astype(numpy.float32))
    rdisp = torch.from_numpy(g.uniform(0.005, 0.02, H * W * 3)
                             .astype(numpy.float32))
    labels = torch.from_numpy(g.integers(0, 1000, n).astype(numpy.int32))
    shuffled = torch.from_numpy(g.permutation(n).astype(numpy.int32))
    return src, mean, rdisp, labels, shuffled


@pytest.mark.parametrize("s,KH,KW,pad,H,W", GEOM)
def test_s2d_conv_equals_strided_conv_cpu(s, KH, KW, pad, H, W):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, H, W, 3, generator=g)
    w = torch.randn(8, KH, KW, 3, generator=g)
    ref = F.conv2d(F.pad(x.permute(0, 3, 1, 2), (pad[0], pad[2], pad[1],
                                                 pad[3])),
                   w.permute(0, 3, 1, 2), stride=s)
    x2 = ops.space_to_depth_ref(x, s, KH, KW, pad)
    w2 = ops._s2d_weights(w, s)
    KH2, KW2 = w2.shape[1], w2.shape[2]
    y = F.conv2d(x2.permute(0, 3, 1, 2), w2.permute(0, 3, 1, 2))
    assert y.shape == ref.shape
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    assert KH2 == -(-KH // s) and KW2 == -(-KW // s)


@pytest.mark.parametrize("s,KH,KW,pad,H,W", GEOM)
def test_fill_minibatch_s2d_reference_cpu(s, KH, KW, pad, H, W):
    src, mean, rdisp, labels, shuffled = _data(7, H, W)
    n, count, start = 5, 4, 2
    plain = torch.zeros(n, H, W, 3)
    lab_a = torch.zeros(n, dtype=torch.int32)
    ops.fill_minibatch(src, shuffled, start, count, plain, mean=mean,
                       rdisp=rdisp, labels=labels, labels_out=lab_a)
    ref = ops.space_to_depth_ref(plain, s, KH, KW, pad)
    H2, W2, C2 = ops.s2d_geometry(src.shape, s, KH, KW, pad)
    out = torch.full((n, H2, W2, C2), 7.0)
    lab_b = torch.zeros(n, dtype=torch.int32)
    idx = torch.zeros(n, dtype=torch.int32)
    m2 = ops.s2d_affine(mean, (H, W, 3), s, KH, KW, pad, 0.0)
    r2 = ops.s2d_affine(rdisp, (H, W, 3), s, KH, KW, pad, 1.0)
    ops.fill_minibatch_s2d(src, shuffled, start, count, out, s, KH, KW, pad,
                           m2, r2, labels=labels, labels_out=lab_b,
                           idx_out=idx)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(lab_a, lab_b)
    assert idx[:count].tolist() == shuffled[start:start + count].tolist()
    assert idx[count:].tolist() == [-1] * (n - count)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 61, 60])
@pytest.mark.parametrize("s,KH,KW,pad,H,W", GEOM)
def test_fill_minibatch_s2d_kernel_matches_fill_then_s2d(s, KH, KW, pad, H,
                                                        W, variant):
    """hvk_fill_minibatch_s2d == hvk_space_to_depth(hvk_fill_minibatch(.))
    bit for bit (same f32 affine map, same bf16 rounding), tail rows of a
    short minibatch zero, labels / indices gathered - for the row-staged
    kernel with four samples per block (default), one sample per block (61)
    and the per-chunk kernel (60)."""
    dev = torch.device("cuda")
    src, mean, rdisp, labels, shuffled = (t.to(dev) for t in _data(13, H, W))
    n, start, count = 11, 1, 9
    plain = torch.zeros(n, H, W, 3, dtype=torch.bfloat16, device=dev)
    la = torch.zeros(n, dtype=torch.int32, device=dev)
    ops.fill_minibatch(src, shuffled, start, count, plain, mean=mean,
                       rdisp=rdisp, labels=labels, labels_out=la)
    ref = ops.space_to_depth(plain, s, KH, KW, pad)
    H2, W2, C2 = ops.s2d_geometry(src.shape, s, KH, KW, pad)
    out = torch.full((n, H2, W2, C2), 3.0, dtype=torch.bfloat16, device=dev)
    lb = torch.zeros(n, dtype=torch.int32, device=dev)
    idx = torch.zeros(n, dtype=torch.int32, device=dev)
    m2 = ops.s2d_affine(mean.cpu(), (H, W, 3), s, KH, KW, pad, 0.0).to(dev)
    r2 = ops.s2d_affine(rdisp.cpu(), (H, W, 3), s, KH, KW, pad, 1.0).to(dev)
    lib = ops._lib.lib()
    try:
        lib.hvk_set_gemm_variant(variant)
        ops.fill_minibatch_s2d(src, shuffled, start, count, out, s, KH, KW,
                               pad, m2, r2, labels=labels, labels_out=lb,
                               idx_out=idx)
        torch.cuda.synchronize()
    finally:
        lib.hvk_set_gemm_variant(-1)
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    assert torch.equal(la, lb)
    assert idx.cpu()[count:].tolist() == [-1] * (n - count)


@pytest.mark.gpu
def test_alexnet_trains_the_same_with_the_fused_s2d_gather():
    """A reduced AlexNet (conv1 11x11 / 4 on 227^2 RGB, LRN, pooling) trained
    with the loader writing conv1's s2d layout follows the run with the
    separate gather + space-to-depth passes."""
    from veles_amd.utils.config import root
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    G = {"learning_rate": 0.01, "gradient_moment": 0.9,
         "weights_decay": 5e-4}
    layers = [
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 11, "ky": 11,
                                    "sliding": 4}, "<-": dict(G)},
        {"type": "norm", "alpha": 1e-4, "beta": 0.75, "n": 5, "k": 2},
        {"type": "max_pooling", "->": {"kx": 3, "ky": 3, "sliding": 2}},
        {"type": "conv_str", "->": {"n_kernels": 64, "kx": 5, "ky": 5,
                                    "padding": 2}, "<-": dict(G)},
        {"type": "max_pooling", "->": {"kx": 3, "ky": 3, "sliding": 2}},
        {"type": "softmax", "->": {"output_sample_shape": 16},
         "<-": dict(G)}]
    res = {}
    old = root.common.engine.fuse_input_layout
    try:
        for fused in (False, True):
            root.common.engine.fuse_input_layout = fused
            random_generator.get().seed(5)
            numpy.random.seed(5)
            torch.manual_seed(0)
            wf = StandardWorkflow(
                DummyLauncher(), loader_name="synthetic_images",
                loader_config={"dataset": "imagenet",
                               "class_lengths": (0, 0, 96),
                               "minibatch_size": 32,
                               "normalization_type": "mean_disp",
                               "n_classes": 16},
                layers=layers, decision_config={"max_epochs": None,
                                                "fail_iterations": None})
            wf.initialize(device=Device(backend="hip"))
            assert (getattr(wf.loader.minibatch_data, "s2d_", None)
                    is not None) == fused
            wf.run_steps(6)
            torch.cuda.synchronize()
            res[fused] = wf.param_store_.master.clone()
    finally:
        root.common.engine.fuse_input_layout = old
    a, b = res[False].float(), res[True].float()
    assert float((a - b).norm() / b.norm()) < 1e-2
