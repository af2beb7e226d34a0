"""Per-device kernel tuning table (``devices/gfx950.json``) and its autotuner.

The reference keeps a per-device JSON of the best GEMM ``BLOCK_SIZE`` /
``VECTOR_OPT`` per dtype and precision level, filled by benchmarking at device
start (``devices/device_infos.json:1-39``, ``veles/backends.py:623-731``
``_fill_device_info_performance_values`` / ``_find_optimal_bs_vo``).  Here the
tile shapes are compile-time (csrc/kernels/gemm.hip), so what is tuned per
device is what the kernels take at run time, per GEMM shape:

* ``wgrad``: the pixel (K) split count of a weight-gradient GEMM (split-K by
  f32 atomics; default :func:`veles_amd.ops.wgrad_splits`, ~512 workgroups);
* ``splitk``: the K split of a low-tile-count GEMM through the f32 workspace
  and its finishing pass (default :func:`veles_amd.ops.auto_splitk`; 0 = no
  split);

plus the ``DeviceBenchmark`` GEMM times per dtype and precision level (the
reference table's own content, ``tools/bench_device.py``).

Shapes come from a real run: ``record()`` logs the geometry of every tunable
call; :func:`tune` replays each one on random operands of the same shape for
every candidate, times them with HIP events (median of ``repeats``) and keeps
the fastest only when it beats the built-in default by more than ``margin``.
The table is read lazily by the ops (``lookup``) from
``root.common.engine.kernels.tuning_file`` / ``VELES_AMD_TUNING_FILE``, else
the in-tree ``devices/<arch>.json``; ``VELES_AMD_TUNING=0`` ignores it.

    python -m veles_amd.ops.autotune --model alexnet --batch 512
"""
from __future__ import annotations

import json
import os
import threading

__all__ = ["TuningTable", "table", "lookup", "record", "recorded", "tune",
           "default_path"]

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
FORMAT = 1


def default_path(arch="gfx950"):
    from veles_amd.utils.config import root, get
    p = os.environ.get("VELES_AMD_TUNING_FILE") or get(
        root.common.engine.kernels.tuning_file, None)
    return p or os.path.join(_REPO, "devices", "%s.json" % arch)


class TuningTable(object):
    """``{"format", "device": {...}, "benchmarks": {...}, "entries":
    {key: {"value", "us", "default", "default_us"}}}`` in one JSON file."""

    def __init__(self, path=None):
        self.path = path or default_path()
        self.data = {"format": FORMAT, "device": {}, "benchmarks": {},
                     "entries": {}}
        self.load()

    def load(self):
        try:
            with open(self.path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            return False
        if not isinstance(d, dict) or d.get("format") != FORMAT or \
                not isinstance(d.get("entries"), dict):
            return False
        self.data = d
        for k in ("device", "benchmarks"):
            self.data.setdefault(k, {})
        return True

    def save(self):
        os.makedirs(os.path.dirname(os.path.abspath(self.path)),
                    exist_ok=True)
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.data, f, indent=1, sort_keys=True)
            f.write("\n")
        os.replace(tmp, self.path)

    @property
    def entries(self):
        return self.data["entries"]

    def get(self, key):
        e = self.entries.get(key)
        return None if e is None else e.get("value")

    def set(self, key, value, us=None, default=None, default_us=None):
        self.entries[key] = {"value": value, "us": us, "default": default,
                             "default_us": default_us}


_TABLE = None
_LOCK = threading.Lock()


def table(reload=False):
    global _TABLE
    with _LOCK:
        if _TABLE is None or reload:
            _TABLE = TuningTable()
        return _TABLE


_ENABLED = os.environ.get("VELES_AMD_TUNING", "1") != "0"


def key(kind, *shape):
    return "%s:%s" % (kind, ":".join(str(int(v)) for v in shape))


def lookup(kind, *shape):
    """Tuned value for a shape, or None (use the built-in default)."""
    if not _ENABLED:
        return None
    return table().get(key(kind, *shape))


# ----------------------------------------------------------------- recording
_LOG = None


def record(on=True):
    """Start (or stop) logging the geometry of every tunable GPU call."""
    global _LOG
    _LOG = {} if on else None


def recorded():
    return dict(_LOG or {})


def log_call(kind, shape, replay):
    """Called by the ops: ``replay`` is the call's geometry (kwargs of the
    replay functions below)."""
    if _LOG is not None:
        _LOG.setdefault(key(kind, *shape), (kind, replay))


# -------------------------------------------------------------------- tuning
def _time(fn, repeats):
    import torch
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(repeats):
        a, b = torch.cuda.Event(enable_timing=True), \
            torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def _wgrad_case(g, dev):
    import torch
    from veles_amd import ops
    x = torch.randn(g["x"], device=dev).to(torch.bfloat16)
    dy = torch.randn(g["dy"], device=dev).to(torch.bfloat16)
    dw = torch.zeros(g["dw"], dtype=torch.float32, device=dev)
    db = torch.zeros(g["dy"][-1], dtype=torch.float32, device=dev)

    def run(sp):
        ops.conv_wgrad(x, dy, dw, g["sliding"], g["padding"], g["groups"],
                       splits=sp, dbias=db)
    return run


def _splitk_case(g, dev):
    import torch
    from veles_amd import ops
    a = torch.randn(g["a"], device=dev).to(torch.bfloat16)
    b = torch.randn(g["b"], device=dev).to(torch.bfloat16)
    out = torch.empty(g["out"], dtype=torch.bfloat16, device=dev)

    def run(sk):
        ops._splitk_forced = sk
        try:
            ops.gemm(a, b, trans_a=g["trans_a"], trans_b=g["trans_b"],
                     out=out)
        finally:
            ops._splitk_forced = None
    return run


def _candidates(kind, default):
    if kind == "wgrad":
        c = {1, 2, 4, 8, 16, 32, 64, 128, 256, default,
             max(1, default // 2), default * 2}
        return sorted(v for v in c if v >= 1)
    return sorted({0, 2, 3, 4, 6, 8, 12, 16, default})


def tune(log=None, repeats=7, margin=0.03, tab=None, verbose=True):
    """Time every candidate of every recorded shape; returns the table."""
    import torch
    tab = tab or table()
    dev = torch.device("cuda", torch.cuda.current_device())
    log = log if log is not None else recorded()
    for k, (kind, g) in sorted(log.items()):
        if kind == "wgrad":
            run = _wgrad_case(g, dev)
        elif kind == "splitk":
            run = _splitk_case(g, dev)
        else:
            continue
        default = int(g["default"])
        times = {c: _time(lambda c=c: run(c), repeats)
                 for c in _candidates(kind, default)}
        best = min(times, key=times.get)
        if times[best] > times[default] * (1.0 - margin):
            best = default
        tab.set(k, int(best), round(times[best], 2), int(default),
                round(times[default], 2))
        if verbose:
            print("%-40s default %-4d %8.1f us -> %-4d %8.1f us" % (
                k, default, times[default], best, times[best]), flush=True)
    return tab


def describe_device(tab=None):
    import torch
    tab = tab or table()
    p = torch.cuda.get_device_properties(torch.cuda.current_device())
    tab.data["device"] = {
        "name": p.name, "arch": getattr(p, "gcnArchName", "gfx950"),
        "compute_units": p.multi_processor_count,
        "memory_gb": round(p.total_memory / 2 ** 30, 1)}
    return tab


def benchmark_device(tab=None, size=3001, repeats=3):
    """The reference table's own measurement: seconds per SIZE^3 GEMM per
    dtype and precision level (``DeviceBenchmark``)."""
    import torch
    from veles_amd import ops
    tab = tab or table()
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}
    for name, dt, levels in (("float", torch.float32, (0, 1, 2)),
                             ("double", torch.float64, (0, 1, 2)),
                             ("bfloat16", torch.bfloat16, (0,))):
        a = torch.rand(size, size, device=dev).to(dt)
        b = torch.rand(size, size, device=dev).to(dt)
        out = torch.empty(size, size, dtype=dt, device=dev)
        for lv in levels:
            kw = {} if dt == torch.bfloat16 else {"precision_level": lv}
            us = _time(lambda: ops.gemm(a, b, out=out, **kw), repeats)
            res.setdefault(name, {})[str(lv)] = {
                "seconds": us * 1e-6, "tflops": 2.0 * size ** 3 / us * 1e-6}
    tab.data["benchmarks"]["gemm_%d" % size] = res
    return tab


def main(argv=None):
    import argparse
    import sys
    sys.path.insert(0, _REPO)
    import veles_amd.ops.autotune as mod
    if mod is not sys.modules[__name__]:
        # run as __main__: the ops log into and read the package module
        return mod.main(argv)
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", action="append", default=None,
                    help="zoo model(s) whose shapes are tuned (alexnet)")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--repeats", type=int, default=7)
    ap.add_argument("--no-device-benchmark", action="store_true")
    a = ap.parse_args(argv)
    os.environ["VELES_AMD_GRAPHS"] = "0"   # record eagerly
    global _ENABLED
    _ENABLED = False                       # record the built-in defaults
    import torch
    from veles_amd.utils.config import root
    root.common.disable.snapshotting = True
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models.zoo import MODELS
    import veles_amd.loader  # noqa: F401
    tab = TuningTable(a.out) if a.out else table()
    dev = Device(backend="hip")
    for model in a.model or ["alexnet"]:
        if model == "none":   # device benchmark only
            continue
        layers_fn, dataset = MODELS[model]
        record(True)
        wf = StandardWorkflow(
            DummyLauncher(), loader_name="synthetic_images",
            loader_config={"dataset": dataset,
                           "class_lengths": (0, 0, 2 * a.batch),
                           "minibatch_size": a.batch,
                           "normalization_type": "mean_disp",
                           "generate_on_device": True},
            layers=layers_fn(), decision_config={"max_epochs": None,
                                                 "fail_iterations": None})
        wf.initialize(device=dev)
        wf.run_steps(1)
        torch.cuda.synchronize()
        log = recorded()
        record(False)
        print("%s b%d: %d tunable shapes" % (model, a.batch, len(log)),
              flush=True)
        tune(log, repeats=a.repeats, tab=tab)
        del wf
        torch.cuda.empty_cache()
    describe_device(tab)
    if not a.no_device_benchmark:
        benchmark_device(tab)
    tab.save()
    print("wrote", tab.path)


if __name__ == "__main__":
    main()
