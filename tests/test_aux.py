"""Auxiliary subsystems: plotting units, publisher, status reporter,
compare_snapshots, callable module, numpy/pickle helpers."""
import json
import os

import numpy
import pytest

import veles_amd
from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import mnist_fc
from veles_amd.utils.config import root
import veles_amd.loader  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wf(tmp_path, epochs=2, snap=True):
    return StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 100, 300),
                       "minibatch_size": 50, "seed": 1},
        layers=mnist_fc(), decision_config={"max_epochs": epochs},
        snapshotter_config={"prefix": "aux", "directory": str(tmp_path),
                            "interval": 1, "time_interval": 0}
        if snap else None)


def test_plotters_and_publisher(tmp_path):
    pytest.importorskip("matplotlib")
    from veles_amd.plotting_units import (
        AccumulatingPlotter, Histogram, ImagePlotter, MatrixPlotter,
        TableMaxMin)
    from veles_amd.publishing import Publisher
    root.common.disable.plotting = False
    wf = _wf(tmp_path, snap=False)
    d = str(tmp_path / "plots")
    err = AccumulatingPlotter(wf, name="valid_err", directory=d,
                              redraw_threshold=0)
    err.link_attrs(wf.decision, ("input", "epoch_n_err_pt"))
    err.input_field = 1
    err.link_from(wf.decision)
    err.gate_skip = ~wf.decision.epoch_ended_flag
    w = ImagePlotter(wf, name="weights", directory=d, redraw_threshold=0,
                     sample_shape=(28, 28), limit=4)
    w.link_attrs(wf.forwards[0], ("input", "weights"))
    w.link_from(wf.decision)
    w.gate_skip = ~wf.decision.epoch_ended_flag
    h = Histogram(wf, name="w_hist", directory=d, redraw_threshold=0)
    h.link_attrs(wf.forwards[1], ("input", "weights"))
    h.link_from(wf.decision)
    m = MatrixPlotter(wf, name="mat", directory=d, redraw_threshold=0)
    m.input = numpy.eye(3)
    t = TableMaxMin(wf, name="table", directory=d, redraw_threshold=0,
                    values={"w0": wf.forwards[0].weights})
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    for u in (m, t):  # not linked into the graph: drive them directly
        u.stopped = False
        u.run()
    for p in (err, w, h, m):
        assert p.files and os.path.getsize(p.files[0]) > 1000, p
    assert len(err.values) == 2
    assert "w0" in open(t.files[0]).read()
    pub = Publisher(wf, output=str(tmp_path / "report.md"))
    pub.publish()
    text = open(tmp_path / "report.md").read()
    assert "## Results" in text and "valid_err.png" in text
    assert "digraph" in text


def test_status_reporter(tmp_path):
    import urllib.request
    from veles_amd.web_status import StatusReporter
    wf = _wf(tmp_path, snap=False)
    rep = StatusReporter(wf, file=str(tmp_path / "st.jsonl"),
                         notification_interval=0, port=0)
    rep.link_from(wf.decision)
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    lines = open(tmp_path / "st.jsonl").read().splitlines()
    assert len(lines) >= 2
    st = json.loads(lines[-1])
    assert st["epoch"] == 2 and "all2all_tanh0" in st["units"]
    got = json.loads(urllib.request.urlopen(
        "http://127.0.0.1:%d/status" % rep.port, timeout=10).read())
    assert got["class"] == "StandardWorkflow"
    rep.stop()


def test_compare_snapshots(tmp_path):
    from veles_amd.scripts.compare_snapshots import compare
    from veles_amd.snapshotter import SnapshotterToFile
    wf = _wf(tmp_path, epochs=3)
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    snaps = sorted(f for f in os.listdir(tmp_path) if "current" not in f)
    assert len(snaps) >= 2
    a = SnapshotterToFile.import_(str(tmp_path / snaps[0]))
    b = SnapshotterToFile.import_(str(tmp_path / snaps[-1]))
    diffs = compare(a, b)
    assert any(u == "all2all_tanh0" and k == "weights" for u, k, _ in diffs)
    assert compare(a, a) == []


def test_callable_module(tmp_path):
    cfg = tmp_path / "cfg.py"
    cfg.write_text(
        "root.mnist_fc.update({'loader_name': 'synthetic_images', "
        "'loader': {'dataset': 'mnist', 'class_lengths': (0, 50, 100), "
        "'minibatch_size': 50}, 'decision': {'max_epochs': 1}})\n"
        "from veles_amd.models.zoo import mnist_fc\n"
        "root.mnist_fc.layers = mnist_fc()\n")
    m = veles_amd(os.path.join(REPO, "samples", "mnist_fc.py"), str(cfg),
                  backend="cpu")
    assert m.workflow.decision.epoch_number == 1
    assert "All2AllTanh" in {c.__name__ for c in veles_amd.__units__}


def test_numpy_ext_and_pickle_helpers():
    import threading
    from veles_amd.utils.numpy_ext import NumDiff, interleave, roundup
    from veles_amd.utils.pickle2 import find_unpicklable
    assert roundup(13, 8) == 16 and roundup(16, 8) == 16
    a = numpy.arange(24).reshape(1, 2, 3, 4)
    assert interleave(a).shape == (1, 3, 4, 2)
    nd = NumDiff()
    assert abs(nd.check_diff(2.0, None, None, lambda x: x ** 3) - 12) < 1e-4

    class Holder(object):
        pass
    h = Holder()
    h.ok = 1
    h.bad = threading.Lock()
    assert find_unpicklable(h) == "obj.bad"
