"""Task-parallel and serving subsystems: genetic optimizer, ensembles,
forward-workflow extraction, RESTful API (reference
veles/genetics, veles/ensemble, veles/restful_api.py)."""
import json
import os
import subprocess
import sys
import threading
import urllib.request

import numpy
import pytest
import torch

from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher
from veles_amd.genetics.core import (
    Population, bin_to_num, gray_decode, gray_encode, num_to_bin)
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import mnist_fc
import veles_amd.loader  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gray_and_binary_codes():
    for n in range(300):
        assert gray_decode(gray_encode(n)) == n
        assert bin(gray_encode(n) ^ gray_encode(n + 1)).count("1") == 1
    b = num_to_bin([0.25, 7], [0, 0], [1, 10], 12, gray=True)
    v = bin_to_num(b, [0, 0], [1, 10], 12, gray=True)
    assert abs(v[0] - 0.25) < 1e-3 and abs(v[1] - 7) < 1e-2


@pytest.mark.parametrize("selection", ["roulette", "tournament", "random"])
def test_population_maximises(selection):
    target = numpy.array([3.0, -1.0])
    pop = Population([-10, -10], [10, 10], 20, seed=5, max_generations=25,
                     selection=selection)
    best = pop.optimize(lambda v: -float(((numpy.array(v) - target) ** 2)
                                         .sum()))
    assert numpy.abs(numpy.array(best.numeric) - target).max() < 1.0
    assert pop.history[-1]["best"] >= pop.history[0]["best"]
    for c in pop:
        assert all(-10 <= x <= 10 for x in c.numeric)


def test_binary_coded_population():
    pop = Population([0, 0], [1, 1], 12, seed=2, max_generations=10,
                     code="gray", bits=10)
    best = pop.optimize(lambda v: -abs(v[0] - 0.7) - abs(v[1] - 0.2))
    assert abs(best.numeric[0] - 0.7) < 0.2


def _trained():
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (60, 100, 300),
                       "minibatch_size": 50, "seed": 1,
                       "normalization_type": "mean_disp"},
        layers=mnist_fc(), decision_config={"max_epochs": 3})
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    return wf


def test_extract_forward_workflow_and_test_mode():
    wf = _trained()
    fw = wf.extract_forward_workflow(loader_config={
        "dataset": "mnist", "class_lengths": (70, 0, 0), "minibatch_size": 32,
        "seed": 1, "normalization_type": "mean_disp"})
    fw.initialize(device=Device(backend="cpu"))
    fw.run()
    r = fw.gather_results()
    out = numpy.array(r["Output"])
    assert out.shape == (70, 10)
    acc = (out.argmax(1) == numpy.asarray(fw.loader.original_labels)).mean()
    assert acc > 0.9
    # the same trained workflow switched to --test mode
    wf.switch_to_testing()
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    r2 = wf.gather_results()
    assert len(r2["Output"]) == 60 and r2["Labels"] == list(range(10))


def test_restful_api_serves_forward_pass():
    from veles_amd.restful_api import RESTfulAPI
    wf = _trained()
    fw = wf.extract_forward_workflow(
        loader_name="restful", loader_config={"minibatch_size": 4},
        result_unit_factory=RESTfulAPI, result_unit_config={"port": 0},
        cyclic=True)
    fw.initialize(device=Device(backend="cpu"))
    api = fw.result_unit
    th = threading.Thread(target=fw.run, daemon=True)
    th.start()
    x = wf.loader.original_data.mem[:3].astype(numpy.float32)
    url = "http://127.0.0.1:%d/service" % api.port
    got = []
    for s in x:
        req = urllib.request.Request(url, data=json.dumps({
            "input": s.tolist(), "codec": "list",
            "shape": list(s.shape)}).encode(),
            headers={"Content-Type": "application/json"})
        got.append(json.loads(urllib.request.urlopen(req, timeout=30)
                              .read()))
    fw.loader.feed(None)
    th.join(30)
    api.stop()
    assert not th.is_alive()
    labels = numpy.asarray(wf.loader.original_labels)[:3]
    assert [g["label"] for g in got] == labels.tolist()
    assert abs(sum(got[0]["result"]) - 1.0) < 1e-4


CFG = """
from veles_amd.genetics.config import Range
root.mnist_fc.update({
    "loader_name": "synthetic_images",
    "loader": {"dataset": "mnist", "class_lengths": (40, 60, 200),
               "minibatch_size": 50, "normalization_type": "mean_disp"},
    "decision": {"max_epochs": 2, "fail_iterations": 20},
    "snapshotter": {"prefix": "tiny", "interval": 1, "time_interval": 0,
                    "directory": %(snap)r},
})
from veles_amd.models.zoo import mnist_fc
root.mnist_fc.layers = mnist_fc(lr=Range(0.1, 0.01, 0.5))
"""


def _cli(args, cwd, timeout=600):
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2")
    return subprocess.run([sys.executable, "-m", "veles_amd"] + args,
                          cwd=cwd, env=env, capture_output=True, text=True,
                          timeout=timeout)


def _setup(tmp_path):
    wf = tmp_path / "mnist_fc.py"
    wf.write_text(open(os.path.join(REPO, "samples", "mnist_fc.py")).read())
    cfg = tmp_path / "mnist_fc_config.py"
    cfg.write_text(CFG % {"snap": str(tmp_path / "snaps")})
    return str(wf), str(cfg)


@pytest.mark.timeout(900)
def test_cli_optimize(tmp_path):
    wf, cfg = _setup(tmp_path)
    res = tmp_path / "opt.json"
    r = _cli([wf, cfg, "-a", "cpu", "--optimize", "3:2", "--result-file",
              str(res)], str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(res.read_text())
    assert len(out["generations"]) == 2
    assert 0 < out["EvaluationFitness"] <= 1
    best = open(tmp_path / "mnist_fc_best_config.py").read()
    assert "learning_rate" in best


@pytest.mark.timeout(900)
def test_cli_ensemble_train_and_test(tmp_path):
    wf, cfg = _setup(tmp_path)
    ens = tmp_path / "ens.json"
    r = _cli([wf, cfg, "-a", "cpu", "--ensemble-train", "2:0.8",
              "--result-file", str(ens)], str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    e = json.loads(ens.read_text())
    assert len(e["models"]) == 2
    assert all(os.path.exists(m["Snapshot"]) for m in e["models"])
    r = _cli([wf, cfg, "-a", "cpu", "--ensemble-test", str(ens)],
             str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    e = json.loads(ens.read_text())
    outs = [numpy.array(m["Output"]) for m in e["models"]]
    assert outs[0].shape == (40, 10)
    from veles_amd.loader import EnsembleLoader
    from veles_amd.dummy import DummyWorkflow
    ld = EnsembleLoader(DummyWorkflow(), file=str(ens), testing=True,
                        minibatch_size=10)
    ld.initialize(device=Device(backend="cpu"))
    assert ld.original_data.mem.shape == (40, 2, 10)


_ = torch


def test_prometheus_text_exposition():
    from veles_amd.web_status import prometheus_text
    st = {"time": 12.5, "rank": 3, "pid": 7, "epoch": 2,
          "last_epoch": {"train_err": 0.25, "ok": True},
          "units": {"conv1": 0.5, 'we"ird': 1.0},
          "device_memory": {"allocated": 1024, "peak": 2048},
          "workflow": "wf"}
    txt = prometheus_text(st)
    assert 'veles_amd_epoch{rank="3"} 2.0' in txt
    assert 'veles_amd_last_epoch_train_err{rank="3"} 0.25' in txt
    assert 'veles_amd_last_epoch_ok{rank="3"} 1.0' in txt
    assert 'veles_amd_device_memory_peak{rank="3"} 2048.0' in txt
    assert 'veles_amd_unit_run_seconds{rank="3",unit="conv1"} 0.5' in txt
    assert "workflow" not in txt and "pid" not in txt
    for line in txt.splitlines():
        assert line.startswith("# TYPE ") or line.startswith("veles_amd_")
