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


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
