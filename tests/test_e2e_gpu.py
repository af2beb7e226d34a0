"""End-to-end numerics of the HIP training step against the float32 CPU
path of the same workflow (the reference's device-vs-numpy pattern,
veles/tests/accelerated_test.py:41-123, applied to whole training steps).

Both runs start from the same weights (host PRNG) and the same synthetic
data (generated on the host), train 5 steps with momentum SGD, and are
compared layer by layer.  The HIP path computes in bf16 (activations,
weights' compute copy, GEMM operands) with f32 accumulation and f32 master
weights; the stated tolerance is therefore on the accumulated UPDATE of
every parameter tensor: ||dW_hip - dW_cpu|| / ||dW_cpu|| <= 0.15, plus the
accumulated training loss of the 5 steps within 5 %.  Dropout is left out (the device and host
draw different mask streams); LRN, grouped convolutions, max pooling, the
fused space-to-depth gather of conv1 and the split-K FC GEMMs are in.
"""
import numpy
import pytest
import torch

from veles_amd.utils.config import root

pytestmark = pytest.mark.gpu


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


def _run(layers, dataset, backend, steps, batch, n_classes=None):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    random_generator.get().seed(77)
    numpy.random.seed(77)
    torch.manual_seed(77)
    cfg = {"dataset": dataset, "class_lengths": (0, 0, batch * steps),
           "minibatch_size": batch, "normalization_type": "mean_disp",
           "seed": 9, "generate_on_device": False}
    if n_classes:
        cfg["n_classes"] = n_classes
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images", loader_config=cfg,
        layers=layers, decision_config={"max_epochs": None,
                                        "fail_iterations": None})
    wf.initialize(device=Device(backend=backend))
    w0 = [f.weights_master.detach().float().cpu().clone()
          for f in wf.forwards if getattr(f, "_pw_", None) is not None]
    wf.run_steps(steps)
    if backend == "hip":
        torch.cuda.synchronize()
    w1 = [f.weights_master.detach().float().cpu().clone()
          for f in wf.forwards if getattr(f, "_pw_", None) is not None]
    m = wf.evaluator.metrics_.detach().float().cpu().clone()
    return w0, w1, m


def _compare(cpu, hip, tol=0.15):
    (c0, c1, cm), (h0, h1, hm) = cpu, hip
    assert len(c0) == len(h0)
    rels = []
    for a0, a1, b0, b1 in zip(c0, c1, h0, h1):
        assert torch.equal(a0, b0), "runs did not start from the same weights"
        dc, dh = a1 - a0, b1 - b0
        rels.append(float((dh - dc).norm() / (dc.norm() + 1e-12)))
    worst = max(rels)
    assert worst <= tol, "per-layer update differences %s (> %.2f)" % (
        ["%.3f" % r for r in rels], tol)
    assert torch.isfinite(hm).all()
    # accumulated TRAIN loss over the 5 steps (metrics[class][1])
    lc, lh = float(cm[2][1]), float(hm[2][1])
    assert abs(lh - lc) <= 0.05 * abs(lc), (lh, lc)
    return worst


def test_lenet_5_steps_hip_matches_fp32_cpu():
    from veles_amd.models.zoo import lenet
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "bfloat16"
    try:
        cpu = _run(lenet(0.01), "mnist", "cpu", 5, 64)
        hip = _run(lenet(0.01), "mnist", "hip", 5, 64)
    finally:
        root.common.engine.precision_type = old
    worst = _compare(cpu, hip)
    print("LeNet: worst relative update difference %.4f" % worst)


def test_reduced_alexnet_5_steps_hip_matches_fp32_cpu():
    old = root.common.engine.precision_type
    root.common.engine.precision_type = "bfloat16"
    try:
        cpu = _run(_small_alexnet(), "imagenet", "cpu", 5, 16, n_classes=16)
        hip = _run(_small_alexnet(), "imagenet", "hip", 5, 16, n_classes=16)
    finally:
        root.common.engine.precision_type = old
    worst = _compare(cpu, hip)
    print("reduced AlexNet: worst relative update difference %.4f" % worst)
