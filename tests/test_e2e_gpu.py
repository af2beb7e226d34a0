"""End-to-end numerics of the HIP training step against the float32 CPU
path of the same workflow (the reference's device-vs-numpy pattern,
veles/tests/accelerated_test.py:41-123, applied to whole training steps).

Both runs start from the same weights (host PRNG) and the same synthetic
data (generated on the host), train 5 steps with momentum SGD, and are
compared layer by layer.  The HIP path computes in bf16 (activations,
weights' compute copy, GEMM operands) with f32 accumulation and f32 master
weights; the tolerance is therefore on the accumulated UPDATE of every
parameter tensor, r = ||dW_hip - dW_cpu|| / ||dW_cpu||, measured against
the bf16 NOISE FLOOR of the same workflow: a third run on the float32 CPU
path that rounds every activation and every back-propagated error to bf16
as the HIP path stores them (nothing else changes).  The HIP run must stay
within 1.25 x that floor + 0.03 for every layer (the first layers of a deep
net sit at r ~ 0.2 from the activation rounding alone: the weight gradient
of conv1 is a sum over 16 x 55 x 55 positions with heavy cancellation), and
the accumulated training loss of the 5 steps within 5 %.  Dropout is left out (the device and host
draw different mask streams); LRN, grouped convolutions, max pooling, the
fused space-to-depth gather of conv1 and the split-K FC GEMMs are in.
"""
import numpy
import pytest
import torch

from veles_amd.utils.config import root



def _small_alexnet():
    g = {"learning_rate": 0.01, "learning_rate_bias": 0.02,
         "gradient_moment": 0.9, "gradient_moment_bias": 0.9,
         "weights_decay": 5e-4, "weights_decay_bias": 0.0}
    lrn = {"n": 5, "alpha": 1e-4 / 5, "beta": 0.75, "k": 1.0}
    pool = {"kx": 3, "ky": 3, "sliding": 2}

    def conv(n, k, s=1, p=0, grp=1):
        return {"type": "conv_str",
                "->": {"n_kernels": n, "kx": k, "ky": k, "sliding": s,
                       "padding": p, "grouping": grp,
                       "weights_filling": "gaussian", "weights_stddev": 0.05,
                       "bias_filling": "constant", "bias_stddev": 0.05},
                "<-": dict(g)}
    return [conv(24, 11, 4), {"type": "norm", "->": dict(lrn)},
            {"type": "max_pooling", "->": dict(pool)},
            conv(64, 5, 1, 2, 2), {"type": "norm", "->": dict(lrn)},
            {"type": "max_pooling", "->": dict(pool)},
            conv(96, 3, 1, 1), conv(96, 3, 1, 1, 2), conv(64, 3, 1, 1, 2),
            {"type": "max_pooling", "->": dict(pool)},
            {"type": "all2all_str",
             "->": {"output_sample_shape": 256, "weights_filling": "gaussian",
                    "weights_stddev": 0.02, "bias_filling": "constant",
                    "bias_stddev": 0.05}, "<-": dict(g)},
            {"type": "softmax",
             "->": {"output_sample_shape": 16, "weights_filling": "gaussian",
                    "weights_stddev": 0.05}, "<-": dict(g)}]


def _round_bf16(arr):
    import numpy as _np
    t = getattr(arr, "mem", None) if arr is not None else None
    if isinstance(t, _np.ndarray) and t.dtype == _np.float32:
        tt = torch.from_numpy(t)
        tt.copy_(tt.bfloat16().float())


def _emulate_bf16_storage(wf):
    """Round each unit's output / err_input to bf16 after it runs."""
    for u in list(wf.forwards) + list(getattr(wf, "gds", [])):
        def run(inner=u.do_run, u=u):
            r = inner()
            _round_bf16(getattr(u, "output", None))
            _round_bf16(getattr(u, "err_input", None))
            return r
        u.__dict__["do_run"] = run


def _run(layers, dataset, backend, steps, batch, n_classes=None,
         bf16_storage=False):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    random_generator.get().seed(77)
    numpy.random.seed(77)
    torch.manual_seed(77)
    # one minibatch more than run: the epoch (and its metrics reset) does
    # not end inside the compared steps
    cfg = {"dataset": dataset, "class_lengths": (0, 0, batch * (steps + 1)),
           "minibatch_size": batch, "normalization_type": "mean_disp",
           "seed": 9, "generate_on_device": False}
    if n_classes:
        cfg["n_classes"] = n_classes
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images", loader_config=cfg,
        layers=layers, decision_config={"max_epochs": None,
                                        "fail_iterations": None})
    wf.initialize(device=Device(backend=backend))
    if bf16_storage:
        _emulate_bf16_storage(wf)
    w0 = [f.weights_master.detach().float().cpu().clone()
          for f in wf.forwards if getattr(f, "_pw_", None) is not None]
    wf.run_steps(steps)
    if backend == "hip":
        torch.cuda.synchronize()
    w1 = [f.weights_master.detach().float().cpu().clone()
          for f in wf.forwards if getattr(f, "_pw_", None) is not None]
    m = wf.evaluator.metrics_.detach().float().cpu().clone()
    return w0, w1, m


def _rel_updates(ref, other):
    (c0, c1, _), (h0, h1, _) = ref, other
    assert len(c0) == len(h0)
    rels = []
    for a0, a1, b0, b1 in zip(c0, c1, h0, h1):
        assert torch.equal(a0, b0), "runs did not start from the same weights"
        dc, dh = a1 - a0, b1 - b0
        rels.append(float((dh - dc).norm() / (dc.norm() + 1e-12)))
    return rels


def _compare(cpu, floor_run, hip):
    rels = _rel_updates(cpu, hip)
    floor = _rel_updates(cpu, floor_run)
    bad = [(i, r, f) for i, (r, f) in enumerate(zip(rels, floor))
           if r > 1.25 * f + 0.03]
    assert not bad, "update differences %s vs bf16 floor %s" % (
        ["%.3f" % r for r in rels], ["%.3f" % f for f in floor])
    hm, cm = hip[2], cpu[2]
    assert torch.isfinite(hm).all()
    # accumulated TRAIN loss over the compared steps (metrics[class][1])
    lc, lh = float(cm[2][1]), float(hm[2][1])
    assert lc > 0
    assert abs(lh - lc) <= 0.05 * abs(lc), (lh, lc)
    return max(rels), max(floor)


@pytest.mark.gpu
def test_lenet_5_steps_hip_matches_fp32_cpu():
    from veles_amd.models.zoo import lenet
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "bfloat16"
    try:
        cpu = _run(lenet(0.01), "mnist", "cpu", 5, 64)
        flo = _run(lenet(0.01), "mnist", "cpu", 5, 64, bf16_storage=True)
        hip = _run(lenet(0.01), "mnist", "hip", 5, 64)
    finally:
        root.common.engine.precision_type = old
    worst, floor = _compare(cpu, flo, hip)
    print("LeNet: worst relative update difference %.4f (bf16 floor %.4f)"
          % (worst, floor))


@pytest.mark.gpu
def test_reduced_alexnet_5_steps_hip_matches_fp32_cpu():
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "bfloat16"
    try:
        cpu = _run(_small_alexnet(), "imagenet", "cpu", 5, 16, n_classes=16)
        flo = _run(_small_alexnet(), "imagenet", "cpu", 5, 16, n_classes=16,
                   bf16_storage=True)
        hip = _run(_small_alexnet(), "imagenet", "hip", 5, 16, n_classes=16)
    finally:
        root.common.engine.precision_type = old
    worst, floor = _compare(cpu, flo, hip)
    print("reduced AlexNet: worst relative update difference %.4f "
          "(bf16 floor %.4f)" % (worst, floor))


def test_bf16_floor_emulation_changes_cpu_updates():
    """CPU check of the floor run itself: it differs from float32, and by
    more in the first layer than in the classifier."""
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "bfloat16"
    try:
        cpu = _run(_small_alexnet(), "imagenet", "cpu", 1, 8, n_classes=16)
        flo = _run(_small_alexnet(), "imagenet", "cpu", 1, 8, n_classes=16,
                   bf16_storage=True)
    finally:
        root.common.engine.precision_type = old
    floor = _rel_updates(cpu, flo)
    assert 0 < floor[-1] < floor[0], floor
