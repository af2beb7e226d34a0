"""HIP-graph capture of the train step (veles_amd/graphs.py) on an MI355X:
the same StandardWorkflow trained with the forward / backward segments
captured and replayed must match the eager run (up to the f32 atomics'
summation order), replays must really advance the device-side dropout seed
and fp8 history, and the host bookkeeping of skipped units must hold."""
import numpy
import pytest
import torch

from veles_amd.utils.config import root

pytestmark = pytest.mark.gpu

G = {"learning_rate": 0.02, "gradient_moment": 0.9, "weights_decay": 1e-4}
LAYERS = [
    {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                "padding": 1}, "<-": dict(G)},
    {"type": "norm", "alpha": 1e-4, "beta": 0.75, "n": 5, "k": 2},
    {"type": "max_pooling", "->": {"kx": 3, "ky": 3, "sliding": 2}},
    {"type": "conv_relu", "->": {"n_kernels": 64, "kx": 3, "ky": 3,
                                 "padding": 1}, "<-": dict(G)},
    {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
    {"type": "all2all_relu", "->": {"output_sample_shape": 256},
     "<-": dict(G)},
    {"type": "dropout", "dropout_ratio": 0.5},
    {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": dict(G)}]


def _train(graphs, steps, precision="bfloat16", layers=LAYERS,
           overlap=True, bucket_mb=32):
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    old = (root.common.engine.graphs, root.common.engine.precision_type,
           root.common.engine.overlap_update, root.common.engine.dp.bucket_mb)
    root.common.engine.graphs = graphs
    root.common.engine.precision_type = precision
    root.common.engine.overlap_update = overlap
    root.common.engine.dp.bucket_mb = bucket_mb
    try:
        random_generator.get().seed(1234)
        numpy.random.seed(1234)
        torch.manual_seed(0)
        wf = StandardWorkflow(
            DummyLauncher(), loader_name="synthetic_images",
            loader_config={"dataset": "mnist", "class_lengths": (0, 128, 640),
                           "minibatch_size": 64, "normalization_type":
                           "mean_disp", "seed": 7, "noise": 110.0},
            layers=layers, decision_config={"max_epochs": None,
                                            "fail_iterations": None})
        wf.initialize(device=Device(backend="hip"))
        wf.run_steps(steps)
        torch.cuda.synchronize()
        return wf
    finally:
        (root.common.engine.graphs, root.common.engine.precision_type,
         root.common.engine.overlap_update,
         root.common.engine.dp.bucket_mb) = old


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _params(wf):
    """{layer/param: master tensor} of every parameterized forward unit."""
    out = {}
    for i, f in enumerate(wf.forwards):
        if getattr(f, "_pw_", None) is None:
            continue
        out["%d.w" % i] = f.weights_master.detach().float().cpu()
        if getattr(f, "_pb_", None) is not None:
            out["%d.b" % i] = f.bias_master.detach().float().cpu()
    return out


def _same_within_spread(got, ref, ref2):
    """Per tensor: ``got`` equals ``ref`` bit for bit when ``ref`` and
    ``ref2`` (the same run twice) agree bit for bit; else |got - ref| stays
    within 4x the run-to-run |ref2 - ref| (plus one fp32 ulp-scale term)."""
    a, b, c = _params(got), _params(ref), _params(ref2)
    assert a.keys() == b.keys() == c.keys()
    for k in b:
        spread = float((c[k] - b[k]).norm())
        diff = float((a[k] - b[k]).norm())
        if spread == 0.0:
            assert torch.equal(a[k], b[k]), "%s: %g" % (k, diff)
        else:
            assert diff <= 4 * spread + 1e-7 * float(b[k].norm()), \
                "%s: %g vs run-to-run %g" % (k, diff, spread)


def test_graphed_training_matches_eager():
    steps = 25  # 2.5 epochs: TRAIN and VALID keys, captures + replays
    eager = _train(False, steps)
    graphed = _train(True, steps)
    assert not getattr(eager, "graph_segments_", [])
    fwd, bwd = graphed.graph_segments_
    # (TRAIN, VALID) / TRAIN, per buffer set of the run-ahead loader
    sets = 2 if getattr(graphed.loader, "_ra_bufs_", None) else 1
    assert fwd.captures == 2 * sets and bwd.captures == sets
    assert fwd.failures == 0 and bwd.failures == 0
    assert bwd.replays >= steps - 4 * sets and fwd.replays >= steps - 4 * sets
    assert graphed.param_store_.steps == eager.param_store_.steps == steps
    # same trajectory (the f32 atomics of split-K / weight gradients sum in
    # a different order run to run: a tolerance, not bit equality)
    assert _rel(graphed.param_store_.master, eager.param_store_.master) < 2e-2
    he, hg = eager.decision.history, graphed.decision.history
    assert len(he) == len(hg) >= 2
    for a, b in zip(he, hg):
        assert abs(a["validation_loss"] - b["validation_loss"]) < \
            0.05 * abs(a["validation_loss"]) + 1e-3
    # the replayed dropout advanced its device seed once per TRAIN step
    from veles_amd import ops
    drop = [u for u in graphed.forwards if type(u).__name__ ==
            "DropoutForward"][0]
    s = drop.seed & 0xFFFFFFFF
    for _ in range(steps):
        s = ops.seed_advance_ref(s)
    assert int(drop.seed_dev_.cpu()[0]) & 0xFFFFFFFF == s


def test_graph_replay_is_faster_for_a_small_step():
    """The point of capture: a small network's step is host-bound eagerly
    (one Python dispatch per kernel); a replay is one graph launch."""
    import time
    small = [dict(LAYERS[0]), LAYERS[2], dict(LAYERS[5]), LAYERS[7]]
    res = {}
    for graphs in (False, True):
        wf = _train(graphs, 6, layers=small)
        wf.run_steps(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wf.run_steps(30)
        torch.cuda.synchronize()
        res[graphs] = time.perf_counter() - t0
    print("eager %.2f ms/step, graphed %.2f ms/step" % (
        res[False] / 30 * 1e3, res[True] / 30 * 1e3))
    assert res[True] < res[False]


def test_graphed_fp8_rolls_the_history():
    from veles_amd.ops import fp8
    steps = 12
    wf = _train(True, steps, precision="float8")
    fwd, bwd = wf.graph_segments_
    assert bwd.replays > 0 and bwd.failures == 0 and fwd.failures == 0
    r = fp8.registry(torch.device("cuda", torch.cuda.current_device()))
    assert int(r.step_dev.cpu()[0]) == r.step


def test_graphed_stochastic_and_input_derivative_units():
    """Units that draw per step (stochastic pooling) or differentiate
    through their input (log / sincos activations) replay correctly: the
    graphed run follows the eager one."""
    layers = [
        {"type": "conv_str", "->": {"n_kernels": 16, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(G)},
        {"type": "stochastic_pooling", "->": {"kx": 2, "ky": 2,
                                              "sliding": 2}},
        {"type": "activation_log"},
        {"type": "all2all_tanh", "->": {"output_sample_shape": 64},
         "<-": dict(G)},
        {"type": "activation_sincos"},
        {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": dict(G)}]
    steps = 15
    eager = _train(False, steps, layers=layers)
    graphed = _train(True, steps, layers=layers)
    fwd, bwd = graphed.graph_segments_
    assert fwd.failures == 0 and bwd.failures == 0 and bwd.replays > 0
    assert _rel(graphed.param_store_.master, eager.param_store_.master) < 2e-2
    sp = graphed.forwards[1]
    assert sp.seed_dev_ is not None


def test_capture_broken_by_a_sync_pins_eager_and_restores_state():
    """A unit that synchronises (.item()) inside the backward capture: the
    capture is abandoned, the stream context is restored (the process does
    not stay on the capture stream), the parameter store's host counters
    are put back before the eager re-run (one step counts once), the key is
    pinned to eager mode, and training matches the eager run."""
    from veles_amd import graphs as G_
    steps = 8
    eager = _train(False, steps)
    seen = {}
    orig_install = G_.install_step_graphs

    def install(wf, warmup=2):
        segs = orig_install(wf, warmup)
        gd = [s for s in segs if s.name == "backward"][0].units[1]
        cls = type(gd)

        def run(self):
            seen["n"] = seen.get("n", 0) + 1
            torch.ones(1, device="cuda").sum().item()  # breaks a capture
            return cls.run(self)
        gd.__class__ = type("Sync" + cls.__name__, (cls,), {"run": run})
        return segs

    G_.install_step_graphs = install
    try:
        base = torch.cuda.current_stream()
        graphed = _train(True, steps)
    finally:
        G_.install_step_graphs = orig_install
    fwd, bwd = graphed.graph_segments_
    assert bwd.failures >= 1 and bwd.captures == 0 and bwd.eager_keys
    assert fwd.failures == 0 and fwd.captures >= 1
    assert torch.cuda.current_stream() == base
    assert graphed.param_store_.steps == eager.param_store_.steps == steps
    assert seen["n"] >= steps
    assert _rel(graphed.param_store_.master, eager.param_store_.master) < 2e-2


@pytest.mark.parametrize("graphs", [False, True])
def test_single_rank_overlapped_update_matches_serial(graphs):
    """One rank, several buckets: each bucket's SGD runs on the side stream
    as soon as its layers' backward is enqueued (ParameterStore
    ._single_overlap), eagerly and inside the captured backward.  Same
    trajectory as the one fused update at the end of the step."""
    steps = 12
    ser = _train(graphs, steps, overlap=False, bucket_mb=0.05)
    ovl = _train(graphs, steps, overlap=True, bucket_mb=0.05)
    st = ovl.param_store_
    assert len(st.buckets) > 2 and st._single is True
    assert ser.param_store_._single is False
    if graphs:
        assert ovl.graph_segments_[1].failures == 0
        assert ovl.graph_segments_[1].replays > 0
    assert st.steps == ser.param_store_.steps == steps
    assert _rel(st.master, ser.param_store_.master) < 2e-2
    assert torch.equal(st.lp, st.master.to(st.lp.dtype))


@pytest.mark.parametrize("graphs", [False, True])
def test_wgrad_side_stream_matches_serial(graphs, monkeypatch):
    """Conv weight gradients on a branch stream (engine.wgrad_stream): they
    run under the backward-data / LRN / pooling kernels below them, eagerly
    and inside the captured backward, and the update waits for the stream.
    Same trajectory as the serial step."""
    steps = 12
    monkeypatch.setenv("VELES_AMD_WGRAD_STREAM", "0")
    ser = _train(graphs, steps, overlap=False)
    ser2 = _train(graphs, steps, overlap=False)
    monkeypatch.setenv("VELES_AMD_WGRAD_STREAM", "1")
    side = _train(graphs, steps, overlap=False)
    assert side.param_store_.branch_grads and \
        not ser.param_store_.branch_grads
    if graphs:
        assert side.graph_segments_[1].failures == 0
        assert side.graph_segments_[1].replays > 0
    assert side.param_store_.steps == ser.param_store_.steps == steps
    # the side stream runs the same kernels on the same operands: bit for
    # bit the serial result when the serial run is itself reproducible, else
    # within the run-to-run spread of its f32-atomic split-K kernels - a race
    # that corrupted a gradient tile would land orders of magnitude above
    # either (the former 2 % whole-vector
    # norm was dominated by the FC weights).  Every parameter tensor of
    # every layer is checked on its own.
    _same_within_spread(side, ser, ser2)
    he, hs = ser.decision.history, side.decision.history
    for a, b in zip(he, hs):
        assert abs(a["validation_loss"] - b["validation_loss"]) < \
            0.05 * abs(a["validation_loss"]) + 1e-3


@pytest.mark.parametrize("graphs", [False, True])
def test_tail_update_matches_serial(graphs, monkeypatch):
    """One rank: the update of every bucket but the last on the side stream
    beside the last layers' weight gradients (engine.tail_update), eagerly
    and inside the captured backward - the same trajectory as one update
    after the backward."""
    steps = 12
    monkeypatch.setenv("VELES_AMD_TAIL_UPDATE", "0")
    ser = _train(graphs, steps, overlap=False, bucket_mb=0.05)
    monkeypatch.setenv("VELES_AMD_TAIL_UPDATE", "1")
    tail = _train(graphs, steps, overlap=False, bucket_mb=0.05)
    assert tail.param_store_._tail and not ser.param_store_._tail
    assert len(tail.param_store_.buckets) > 1
    if graphs:
        assert tail.graph_segments_[1].failures == 0
        assert tail.graph_segments_[1].replays > 0
    assert tail.param_store_.steps == ser.param_store_.steps == steps
    assert _rel(tail.param_store_.master, ser.param_store_.master) < 2e-2
    st = tail.param_store_
    assert torch.equal(st.lp, st.master.to(st.lp.dtype))


def _solo_run(out, solo, steps, port):
    import os
    import numpy
    import torch
    os.environ["VELES_AMD_DP_SOLO_COLLECTIVES"] = "1" if solo else "0"
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    from veles_amd.utils.config import root
    root.common.disable.snapshotting = True
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models.zoo import lenet
    from veles_amd.parallel.dp import DataParallel
    import veles_amd.loader  # noqa: F401
    dp = DataParallel(backend="nccl")
    la = DummyLauncher()
    la.dp_ = dp
    wf = StandardWorkflow(
        la, loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 0, 2560),
                       "minibatch_size": 256,
                       "normalization_type": "mean_disp", "seed": 4},
        layers=lenet(0.01), decision_config={"max_epochs": None,
                                             "fail_iterations": None})
    wf.initialize(device=Device(backend="hip"))
    wf.run_steps(steps)
    torch.cuda.synchronize()
    segs = {s.name: (s.captures, s.replays) for s in wf.graph_segments_}
    w = [f.weights_master.float().cpu().numpy().copy() for f in wf.forwards
         if getattr(f, "_pw_", None) is not None]
    numpy.savez(out, *w)
    with open(out + ".json", "w") as f:
        import json
        json.dump({"segs": segs, "multi": bool(dp.multi),
                   "graph_safe": bool(wf.param_store_.graph_safe())}, f)
    dp.shutdown()


@pytest.mark.gpu
def test_solo_rccl_path_captures_backward_and_matches_dp1(tmp_path):
    """The multi-rank step through a one-rank RCCL process group
    (VELES_AMD_DP_SOLO_COLLECTIVES=1): bucketed all-reduces and per-bucket
    updates on the side stream, all captured in the backward HIP graph and
    replayed - ends 6 steps with the weights of the plain single-GPU step
    (split-K atomics make runs differ in the last bits only)."""
    import json
    import socket
    import numpy
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    res = {}
    for solo in (True, False):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        out = str(tmp_path / ("solo%d.npz" % solo))
        p = ctx.Process(target=_solo_run, args=(out, solo, 6, port))
        p.start()
        p.join(300)
        assert p.exitcode == 0
        res[solo] = (numpy.load(out), json.load(open(out + ".json")))
    (ws, js), (wp, jp) = res[True], res[False]
    assert js["multi"] and js["graph_safe"]
    assert not jp["multi"]
    cap, rep = js["segs"]["backward"]
    assert cap == 1 and rep >= 2, js["segs"]
    for k in ws.files:
        assert numpy.isfinite(ws[k]).all()
        numpy.testing.assert_allclose(ws[k], wp[k], rtol=1e-4, atol=1e-6)


def _runahead_run(on, steps, at="backward"):
    import os
    os.environ["VELES_AMD_LOADER_RUNAHEAD"] = "1" if on else "0"   # opt-in
    os.environ["VELES_AMD_LOADER_RUNAHEAD_AT"] = at
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.prng import random_generator
    from test_e2e_gpu import _small_alexnet
    import veles_amd.loader  # noqa: F401
    random_generator.get().seed(21)
    torch.manual_seed(21)
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "imagenet", "n_classes": 16,
                       "class_lengths": (0, 0, 96), "minibatch_size": 32,
                       "normalization_type": "mean_disp", "seed": 5},
        layers=_small_alexnet(), decision_config={"max_epochs": None,
                                                  "fail_iterations": None},
        graph_warmup=1)
    wf.initialize(device=Device(backend="hip"))
    wf.run_steps(steps)
    torch.cuda.synchronize()
    ld = wf.loader
    assert ld.runahead_anchor_ is wf.gds[-1]   # the first backward unit
    w = [f.weights_master.float().cpu().clone() for f in wf.forwards
         if getattr(f, "_pw_", None) is not None]
    segs = {s.name: (s.captures, s.replays) for s in wf.graph_segments_}
    return w, ld.runahead_hits, ld.runahead_misses, segs


@pytest.mark.parametrize("at", ["backward", "fill"])
def test_loader_runahead_matches_serial_gather(at):
    """The double-buffered gather (the next minibatch's fill on a side
    stream, launched as the backward starts or right after this step's
    fill; forward / backward graphs keyed by buffer parity) trains like
    the serial gather over 3 epochs of 3 minibatches (every epoch end is a
    reshuffle: a prediction miss), with the space-to-depth conv1 input."""
    import os
    names = ("VELES_AMD_LOADER_RUNAHEAD", "VELES_AMD_LOADER_RUNAHEAD_AT")
    old = {n: os.environ.get(n) for n in names}
    try:
        ws, _, _, _ = _runahead_run(False, 9)
        wr, hits, misses, segs = _runahead_run(True, 9, at)
    finally:
        for n in names:
            if old[n] is None:
                os.environ.pop(n, None)
            else:
                os.environ[n] = old[n]
    assert hits >= 5 and misses >= 2, (hits, misses)
    assert segs["forward"][0] == 2, segs   # one graph per buffer set
    for a, b in zip(ws, wr):
        assert torch.isfinite(b).all()
        # split-K atomics: the runs differ in the last bits, not by a step
        assert _rel(b, a) < 2e-3
