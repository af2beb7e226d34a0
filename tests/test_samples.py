"""The BASELINE.json sample workflows (samples/*.py) load and initialize
through the CLI (``python -m veles_amd wf.py - --dry-run``), and the small
ones train an epoch on the CPU device."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cli(*args, timeout=600):
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "veles_amd"] + list(args),
                       cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return r.stdout + r.stderr


@pytest.mark.parametrize("name", ["mnist_conv", "cifar_conv"])
def test_sample_trains_one_epoch_cpu(name):
    out = cli("samples/%s.py" % name, "-", "-a", "cpu",
              "root.%s.decision.max_epochs=1" % name,
              "root.%s.loader.class_lengths=(0, 200, 400)" % name,
              "root.common.disable.snapshotting=True")
    assert "Workflow wall time" in out


@pytest.mark.parametrize("name", ["alexnet", "vgg16"])
def test_big_sample_loads_cpu(name):
    cli("samples/%s.py" % name, "-", "-a", "cpu", "--dry-run", "init")


def test_cli_html_help_and_plot_switches():
    out = cli("--html-help")
    assert out.lstrip().startswith("<!DOCTYPE html>")
    assert "--master-addr" in out and "--no-graphics-client" in out
    out = cli("samples/mnist_conv.py", "-", "-a", "cpu", "--dry-run", "load",
              "--no-graphics-client", "-p", "", "--dump-config")
    assert "plotting" in out
