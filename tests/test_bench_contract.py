"""bench.py's driver contract on the multi-rank path, rehearsed on the CPU:
the driver's own launcher (`torch.distributed.run --nnodes=1 --nproc-per-node
N --master-addr 127.0.0.1`), gloo instead of RCCL, AlexNet at a tiny batch.
Rank 0 prints exactly ONE JSON line; value is the whole-job rate over all
ranks (global batch / max-over-ranks step time)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(600)
def test_bench_two_ranks_one_json_line():
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--cpu", "--batch", "4",
           "--steps-per-epoch", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
              "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
              "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    c = d["config"]
    assert c["model"] == "alexnet" and c["parallelism"] == "dp2"
    assert c["global_batch"] == 8 and c["per_gpu_batch"] == 4
    assert c["dp"]["world_size_seen"] == 2
    # whole-job samples/s from the max-over-ranks step time
    assert d["ms_per_step"] > 0
    assert d["value"] == pytest.approx(8 / (d["ms_per_step"] / 1e3),
                                       rel=0.02)
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]


@pytest.mark.timeout(600)
def test_bench_spawns_ranks_without_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE spawns the two ranks
    itself (parallel/launch.spawn_ranks) and reports n_gpus 2 - never a
    one-rank line for --gpus 2."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--cpu", "--batch", "4", "--steps-per-epoch",
           "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    c = d["config"]
    assert c["parallelism"] == "dp2" and c["dp"]["world_size_seen"] == 2
    # every rank's graph state is reported (gloo keeps the backward eager)
    rows = c["dp"]["per_rank_graphs"]
    assert [r_[0] for r_ in rows] == [0, 1]
    assert all(r_[1] == 0 for r_ in rows)


@pytest.mark.timeout(600)
def test_bench_watchdog_ends_a_stalled_rank():
    """A rank that stops making progress (as one stuck in a collective
    would) trips the N > 1 step watchdog: the job exits non-zero with a
    [watchdog] line instead of hanging."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", VELES_AMD_BENCH_STALL_RANK="1",
               VELES_AMD_BENCH_WATCHDOG_S="8")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--cpu", "--batch", "4", "--steps-per-epoch",
           "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=540)
    assert r.returncode != 0
    assert "[watchdog]" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(600)
def test_bench_watchdog_default_bound_is_well_under_driver_timeout():
    """With the DEFAULT settings a rank that stalls after its warmup is
    ended by its own watchdog (armed by the first finished step) in about
    a minute - long before the driver's 600 s limit on the whole command."""
    import time
    sys.path.insert(0, ROOT)
    import bench
    assert bench.WATCHDOG_STEP_S <= 120 and bench.WATCHDOG_INIT_S < 600
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                        "VELES_AMD_BENCH_WATCHDOG_S",
                        "VELES_AMD_BENCH_WATCHDOG_INIT_S")}
    env.update(OMP_NUM_THREADS="2", VELES_AMD_BENCH_STALL_RANK="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--cpu", "--batch", "4", "--steps-per-epoch",
           "2"]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=540)
    dt = time.time() - t0
    assert r.returncode != 0
    assert "[watchdog]" in r.stderr and "before the first step" not in \
        r.stderr, r.stderr[-3000:]
    assert dt < 240, dt


def test_watchdog_arms_on_first_step():
    """init_timeout covers the start; the short per-step bound applies only
    once a step has finished."""
    import threading
    import time
    from veles_amd.parallel.faults import Watchdog
    fired = threading.Event()
    wd = Watchdog(0.3, on_expire=fired.set, init_timeout=30).start()
    time.sleep(1.0)
    assert not fired.is_set() and not wd.armed
    wd.kick()
    assert wd.armed
    assert fired.wait(5.0)
    wd.stop()
    fired2 = threading.Event()
    wd2 = Watchdog(30, on_expire=fired2.set, init_timeout=0.3).start()
    assert fired2.wait(5.0)
    wd2.stop()


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_watchdog_and_fault_hooks_fire_on_a_real_workflow():
    """The hooks sit on the decision unit's scheduled dispatch (do_run),
    not only on a direct run() call: a real workflow kicks once per step."""
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models.zoo import mnist_fc
    from veles_amd.parallel.faults import FaultInjector, Watchdog
    import veles_amd.loader  # noqa: F401
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 0, 200),
                       "minibatch_size": 50},
        layers=mnist_fc(), decision_config={"max_epochs": None,
                                            "fail_iterations": None})
    wf.initialize(device=Device(backend="cpu"))
    wd = Watchdog(1000.0, init_timeout=1000.0).install(wf)
    inj = FaultInjector(wf, 0.0).install()
    draws = []
    rng = inj.rng.random
    inj.rng.random = lambda: draws.append(1) or rng()
    wf.run_steps(3)
    wd.stop()
    assert wd.kicks == 3 and wd.armed
    assert len(draws) == 3
