"""Exact resume on the GPU training paths (reference
veles/units.py:859-885 and veles/snapshotter.py:387-420: every generator's
state is saved and the whole workflow pickled so that a restored run
continues the same trajectory).

A workflow trains k steps, is pickled exactly as the snapshotter pickles it
(``pickle.dumps(workflow)``), restored into a fresh workflow object,
re-initialised on the device and trained m more steps.  Its master weights
must equal those of an uninterrupted k + m run bit for bit, in the
deterministic mode (``ops.set_deterministic``: no f32-atomic reductions;
two uninterrupted runs are checked to be bit-identical first).  The
device-resident state that transient attributes used to drop is covered:

* the dropout / stochastic-pooling seed sequence (``seed_dev_``, advanced on
  the device every step, ``veles_amd/prng/device_seed.py``);
* the fp8 delayed-scaling state (amax histories, shards, primed flags and
  the registry's roll counter, ``fp8.Scaler.state_dict``).

A control run restores WITHOUT the device seed (the pre-round-6 behaviour)
and must land far from the uninterrupted run: the comparison has the power
to see a lost mask stream.  Eager and HIP-graph replay both."""
import pickle

import numpy
import pytest
import torch

from veles_amd.utils.config import root

G = {"learning_rate": 0.01, "learning_rate_bias": 0.02,
     "gradient_moment": 0.9, "gradient_moment_bias": 0.9,
     "weights_decay": 5e-4, "weights_decay_bias": 0.0}


def _alexnet_dropout():
    """Reduced AlexNet (s2d conv1, LRN, grouped convs, pools) with a
    dropout after each of its two fully-connected layers."""
    lrn = {"n": 5, "alpha": 1e-4 / 5, "beta": 0.75, "k": 1.0}
    pool = {"kx": 3, "ky": 3, "sliding": 2}

    def conv(n, k, s=1, p=0, grp=1):
        return {"type": "conv_str",
                "->": {"n_kernels": n, "kx": k, "ky": k, "sliding": s,
                       "padding": p, "grouping": grp,
                       "weights_filling": "gaussian", "weights_stddev": 0.05,
                       "bias_filling": "constant", "bias_stddev": 0.05},
                "<-": dict(G)}

    def fc(n):
        return {"type": "all2all_str",
                "->": {"output_sample_shape": n, "weights_filling": "gaussian",
                       "weights_stddev": 0.02, "bias_filling": "constant",
                       "bias_stddev": 0.05}, "<-": dict(G)}
    return [conv(24, 11, 4), {"type": "norm", "->": dict(lrn)},
            {"type": "max_pooling", "->": dict(pool)},
            conv(64, 5, 1, 2, 2), {"type": "norm", "->": dict(lrn)},
            {"type": "max_pooling", "->": dict(pool)},
            conv(96, 3, 1, 1), conv(96, 3, 1, 1, 2), conv(64, 3, 1, 1, 2),
            {"type": "max_pooling", "->": dict(pool)},
            fc(256), {"type": "dropout", "->": {"dropout_ratio": 0.5}},
            fc(256), {"type": "dropout", "->": {"dropout_ratio": 0.5}},
            {"type": "softmax",
             "->": {"output_sample_shape": 16, "weights_filling": "gaussian",
                    "weights_stddev": 0.05}, "<-": dict(G)}]


def _fp8_vgg_dropout():
    """A small VGG-style fp8 stack (3x3 convs, 2x2 pools) with an
    fully-connected layer and dropout before the classifier."""
    def conv(n):
        return {"type": "conv_str",
                "->": {"n_kernels": n, "kx": 3, "ky": 3, "padding": 1,
                       "weights_filling": "gaussian",
                       "weights_stddev": 0.05}, "<-": dict(G)}
    pool = {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}}
    return [conv(32), conv(32), dict(pool), conv(64), conv(64), dict(pool),
            {"type": "all2all_str", "->": {"output_sample_shape": 256,
                                           "weights_filling": "gaussian",
                                           "weights_stddev": 0.02},
             "<-": dict(G)},
            {"type": "dropout", "->": {"dropout_ratio": 0.5}},
            {"type": "softmax", "->": {"output_sample_shape": 10},
             "<-": dict(G)}]


def _make(layers, dataset, backend, batch, n_batches, n_classes=None):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    from veles_amd.ops import fp8
    import veles_amd.loader  # noqa: F401
    # a fresh scaler registry per run: its roll counter (the history slot
    # the next roll writes) is per process, as in a real job
    fp8._REGISTRIES.clear()
    random_generator.get().seed(31)
    numpy.random.seed(31)
    torch.manual_seed(31)
    cfg = {"dataset": dataset, "class_lengths": (0, 0, batch * n_batches),
           "minibatch_size": batch, "normalization_type": "mean_disp",
           "seed": 5, "generate_on_device": False}
    if n_classes:
        cfg["n_classes"] = n_classes
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images", loader_config=cfg,
        layers=layers, decision_config={"max_epochs": None,
                                        "fail_iterations": None})
    wf.initialize(device=Device(backend=backend))
    return wf


def _master(wf):
    if wf.param_store_.master.is_cuda:
        torch.cuda.synchronize()
    return wf.param_store_.master.detach().float().cpu().clone()


def _resumed(layers, dataset, backend, batch, k, m, n_classes=None,
             drop_seed=False):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    wf = _make(layers, dataset, backend, batch, k + m + 1, n_classes)
    wf.run_steps(k)
    blob = pickle.dumps(wf, protocol=pickle.HIGHEST_PROTOCOL)
    del wf
    wf2 = pickle.loads(blob)
    if drop_seed:   # the pre-round-6 behaviour: the device seed re-drawn
        for u in wf2:
            if hasattr(u, "seed_dev_saved"):
                u.seed_dev_saved = None
    wf2.workflow = DummyLauncher()
    wf2.initialize(device=Device(backend=backend))
    wf2.run_steps(m)
    return wf2


def _check(layers, dataset, backend, batch, k, m, n_classes=None,
           control=True):
    # deterministic mode (ops.set_deterministic): no f32-atomic reductions
    # in the gradient path, so two uninterrupted runs are bit-identical and
    # the resumed run must be too
    from veles_amd import ops
    ops.set_deterministic(True)
    try:
        ref = _master(_run_through(layers, dataset, backend, batch, k + m,
                                   n_classes))
        ref2 = _master(_run_through(layers, dataset, backend, batch, k + m,
                                    n_classes))
        got = _master(_resumed(layers, dataset, backend, batch, k, m,
                               n_classes))
        bad = _master(_resumed(layers, dataset, backend, batch, k, m,
                               n_classes, drop_seed=True)) if control \
            else None
    finally:
        ops.set_deterministic(False)
    spread = float((ref2 - ref).norm())
    diff = float((got - ref).norm())
    scale = float(ref.norm())
    assert torch.isfinite(got).all()
    assert spread == 0.0, "deterministic mode is not: run-to-run %g" % spread
    assert torch.equal(got, ref), \
        "resumed run differs from the uninterrupted one: %g" % diff
    if control:
        lost = float((bad - ref).norm())
        assert lost > 100.0 * max(diff, spread, 1e-9 * scale), \
            "control without the device seed is not distinguishable: " \
            "%g vs %g" % (lost, diff)
    return diff, spread


def _run_through(layers, dataset, backend, batch, steps, n_classes=None):
    wf = _make(layers, dataset, backend, batch, steps + 1, n_classes)
    wf.run_steps(steps)
    return wf


def _with(graphs, precision, fn):
    old = (root.common.engine.graphs, root.common.engine.precision_type)
    root.common.engine.graphs = graphs
    root.common.engine.precision_type = precision
    try:
        return fn()
    finally:
        (root.common.engine.graphs,
         root.common.engine.precision_type) = old


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_alexnet_dropout_resume_exact_gpu(graphs):
    d, s = _with(graphs, "bfloat16", lambda: _check(
        _alexnet_dropout(), "imagenet", "hip", 16, 3, 3, n_classes=16))
    print("AlexNet+dropout resume: diff %g, run-to-run spread %g" % (d, s))


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_fp8_vgg_dropout_resume_exact_gpu(graphs):
    d, s = _with(graphs, "float8", lambda: _check(
        _fp8_vgg_dropout(), "cifar10", "hip", 32, 3, 3))
    print("fp8 VGG-style resume: diff %g, run-to-run spread %g" % (d, s))


def test_fp8_and_dropout_resume_exact_cpu():
    """CPU: the fp8 scaler state and the dropout / host generators go
    through the pickle and the resumed float8 run is bit-identical."""
    def run():
        ref = _master(_run_through(_fp8_vgg_dropout(), "cifar10", "cpu", 8,
                                   4))
        got = _master(_resumed(_fp8_vgg_dropout(), "cifar10", "cpu", 8, 2, 2))
        return ref, got
    ref, got = _with(False, "float8", run)
    assert torch.equal(ref, got)


def test_scaler_state_roundtrip_cpu():
    from veles_amd.ops import fp8
    s = fp8.Scaler("cpu", fp8.E5M2)
    x = torch.randn(64) * 3
    fp8.quantize(x, s)
    s.registry.roll()
    fp8.quantize(x * 2, s)
    d = pickle.loads(pickle.dumps(s.state_dict()))
    t = fp8.Scaler("cpu", fp8.E5M2)
    step = s.registry.step
    s.registry.step = 0
    t.load_state_dict(d)
    assert t.primed and s.registry.step == step
    assert torch.equal(t.state, s.state) and torch.equal(t.shard, s.shard)
    assert t.scale() == s.scale()
    with pytest.raises(ValueError):
        fp8.Scaler("cpu", fp8.E4M3).load_state_dict(d)


def test_device_seed_save_get_cpu_tensor():
    from veles_amd.prng import device_seed

    class U(object):
        seed_dev_ = None
    u = U()
    draws = []
    sd = device_seed.get(u, torch.device("cpu"),
                         lambda: draws.append(1) or 1234)
    assert int(sd[0]) == 1234 and draws == [1]
    sd.add_(7)
    device_seed.save(u)
    assert u.seed_dev_saved == 1241
    v = U()
    v.seed_dev_saved = u.seed_dev_saved
    sd2 = device_seed.get(v, torch.device("cpu"), lambda: 1 / 0)
    assert int(sd2[0]) == 1241 and v.seed_dev_saved is None
