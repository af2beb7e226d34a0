#!/usr/bin/env python3
"""Headline benchmark: AlexNet-ImageNet training throughput (samples/s for the
whole node), bf16, synthetic data, random-init weights, synchronous data
parallelism over RCCL (one process per MI355X).

    python bench.py --gpus N --steps K --warmup W [--batch B]

For N > 1 the driver launches it under torch.distributed.run (one rank per
GPU).  Started with --gpus N > 1 and no WORLD_SIZE, it spawns the N ranks
itself (veles_amd.parallel.launch.spawn_ranks, from a parent that makes no
GPU call) and exits with the group's code; it never reports a 1-rank result
for --gpus N.  At N > 1 every rank runs a step watchdog
(veles_amd.parallel.faults.Watchdog): a rank that makes no progress for
VELES_AMD_BENCH_WATCHDOG_S seconds (default 60) once its first step has
finished, or that reaches no first step within
VELES_AMD_BENCH_WATCHDOG_INIT_S seconds (default 300) - e.g. a collective
whose peer never arrives - prints a [watchdog] line and exits 124.  Every timed step is a full training step through the veles_amd
StandardWorkflow: device minibatch gather + normalisation, forward, softmax
evaluator, decision, backward, bucketed gradient all-reduce, fused SGD.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = ("samples/sec (whole node) AlexNet-ImageNet training at "
                   "1/2/4/8 MI355X")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # 3072 per GPU (end of round 5, profiles/r5/alexnet_batch_sweep_r5t.log:
    # b2048 179.8-180.3k, b3072 184.5-186.0k, b4096 184.5-186.3k, b6144
    # 185.9k img/s on one MI355X; round 4: b2048 154.3k, b3072 156.2k): the
    # smallest batch on the plateau, ~30 GB of the 288 GB HBM with every
    # activation tensor under 2 GB (the 32-bit buffer offsets of the LDS-DMA
    # loaders; b4096's conv1 output is 2.4 GB and runs image-chunked, b8192
    # passes the LRN kernels' 2^31-element limit), and 1.5x the compute per
    # all-reduce of b2048 for the multi-GPU points
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU minibatch (weak scaling); default 3072, "
                         "512 for vgg16 (the fp8 and bf16 throughput "
                         "plateau: profiles/r4/vgg16_batch_sweep.md)")
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--precision", default="bfloat16",
                    choices=("bfloat16", "float8"),
                    help="float8: e4m3/e5m2 MFMA for conv and FC forward + "
                         "backward-data (BASELINE config 5, VGG-16)")
    ap.add_argument("--steps-per-epoch", type=int, default=16)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--profile-json", default=None)
    ap.add_argument("--stats-steps", type=int, default=3,
                    help="N > 1: untimed eager steps after the timed ones "
                         "that record the per-bucket all-reduce timeline")
    ap.add_argument("--mark-steps", action="store_true",
                    help="bracket the timed steps with hvk_trace_marker "
                         "kernels (step-only rocprofv3 summaries)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 512 if args.model == "vgg16" else 3072
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn(args)

    import torch
    from veles_amd.utils.config import root
    root.common.disable.snapshotting = True
    root.common.engine.precision_type = args.precision
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models.zoo import MODELS
    from veles_amd.parallel.dp import DataParallel
    import veles_amd.loader  # noqa: F401 (registers loaders)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world),
              file=sys.stderr)
        return 2
    backend = "cpu" if args.cpu or not torch.cuda.is_available() else "hip"
    # exposed all-reduce wait per step (models/params.py comm_report)
    os.environ.setdefault("VELES_AMD_DP_STATS", "1")
    # VELES_AMD_DP_BACKEND=gloo rehearses the multi-rank path with several
    # ranks on one GPU (RCCL refuses two ranks on one device)
    dp = DataParallel(backend=os.environ.get("VELES_AMD_DP_BACKEND") or
                      ("gloo" if backend == "cpu" else "nccl"))
    if backend == "hip":
        torch.cuda.set_device(dp.local_rank % torch.cuda.device_count())
    device = Device(backend=backend)
    layers_fn, dataset = MODELS[args.model]
    global_batch = args.batch * dp.world_size
    # the resident synthetic set: --steps-per-epoch minibatches of ONE
    # rank's batch, at least one global minibatch.  Every rank holds the
    # whole set (the global shuffle may hand any sample to any rank), so the
    # per-rank HBM it takes is fixed up to N = steps_per_epoch (16: 49152
    # images, 7.6 GB at b3072) and grows linearly past it; an epoch of one or
    # two steps measured as cheap as sixteen (152.9k vs 154.3k img/s at
    # b2048, profiles/r4/alexnet_batch_sweep.md)
    n_train = max(global_batch, args.batch * args.steps_per_epoch)
    launcher = DummyLauncher()
    launcher.dp_ = dp
    wf = StandardWorkflow(
        launcher, loader_name="synthetic_images",
        loader_config={"dataset": dataset, "class_lengths": (0, 0, n_train),
                       "minibatch_size": global_batch,
                       "normalization_type": "mean_disp",
                       "generate_on_device": backend == "hip"},
        layers=layers_fn(), decision_config={"max_epochs": None,
                                             "fail_iterations": None},
        # capture the forward / backward segments inside the warmup steps,
        # after two eager passes (buffers a unit allocates lazily on its
        # second pass would otherwise be zero-filled inside the captured
        # graph, i.e. on every replay); the run-ahead loader alternates two
        # buffer sets, one graph each, so each set needs its passes
        graph_warmup=_graph_warmup(args.warmup))
    wf.initialize(device=device)
    wd = _watchdog(wf, dp)

    def sync():
        if backend == "hip":
            torch.cuda.synchronize()

    wf.run_steps(args.warmup)
    sync()
    _stall_for_test(dp)
    store = getattr(wf, "param_store_", None)
    if store is not None:
        store.comm_report()   # drop the warmup steps' events
    dp.barrier()
    sync()
    mark = args.mark_steps and backend == "hip"
    if mark:
        from veles_amd import ops
        ops.trace_marker(1, device.stream())
    t0 = time.perf_counter()
    wf.run_steps(args.steps)
    if mark:
        ops.trace_marker(2, device.stream())
    sync()
    dp.barrier()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    if dp.world_size > 1:
        if backend == "hip":
            t = t.cuda()
        dp.all_reduce_max(t)
    dt = float(t.cpu()[0])
    value = args.steps * global_batch / dt
    if dp.multi and store is not None:
        # untimed instrumented steps after the timed region: eager passes
        # with per-bucket events (a captured backward records none)
        from veles_amd import graphs
        store.comm_report()
        store.timeline_report()
        with graphs.suspended():
            wf.run_steps(args.stats_steps)
        sync()
    dp_info = dp_report(dp, store, backend, wf)
    if dp.rank == 0:
        base = None
        try:
            with open(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                   "BASELINE.json")) as f:
                base = json.load(f).get("published", {}).get("value")
        except Exception:
            base = None
        shape = "x".join(str(v) for v in wf.loader.sample_shape)
        metric = BASELINE_METRIC if args.model == "alexnet" else \
            "samples/sec (whole node) %s training" % args.model
        out = {"metric": metric, "value": round(value, 2),
               "unit": "samples/s", "n_gpus": dp.world_size,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak",
               "vs_baseline": (value / base) if base else None,
               "dtype": ("fp8" if args.precision == "float8" else "bf16")
               if backend == "hip" else "fp32",
               "data": "synthetic (uint8 %s images resident in HBM, "
                       "random-init weights)" % shape,
               "config": {"model": args.model, "global_batch": global_batch,
                          "per_gpu_batch": args.batch, "seq_len": None,
                          "parallelism": "dp%d" % dp.world_size,
                          "image": shape,
                          "grad_allreduce": dp_info.pop("grad_allreduce"),
                          "dp": dp_info,
                          "hip_graphs": [
                              "%s:%d captured/%d replayed" % (
                                  s.name, s.captures, s.replays)
                              for s in getattr(wf, "graph_segments_", [])]}}
        print(json.dumps(out), flush=True)
        if args.profile_json:
            with open(args.profile_json, "w") as f:
                stats = [(u.name, t_, n) for u, t_, n in
                         wf.get_unit_run_time_stats()]
                json.dump({"result": out, "unit_stats": stats}, f, indent=1)
    dp.barrier()
    if wd is not None:
        wd.stop()
    dp.shutdown()
    return 0


def _spawn(args):
    """--gpus N without a launcher: one child rank per GPU (the driver's
    torch.distributed.run contract: RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), rank 0's JSON line on this
    process's stdout.  This parent never touches the GPU."""
    from veles_amd.parallel.launch import spawn_ranks
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    code = spawn_ranks(list(range(args.gpus)), cmd)
    if code:
        print("bench.py: rank group exited with %s" % code, file=sys.stderr)
    return code


# the hang bounds (seconds): per step once the first step has finished
# (a step takes ~17 ms at b3072; the longest legitimate gap between two
# decision runs is a warmup step with its HIP-graph capture, a few
# seconds), and from the watchdog's start to the first finished step.
# Both sit well below the driver's 600 s limit on the whole command, so a
# hung collective is reported by the rank itself (reference: the master
# drops a slave after max(mean + 3 sigma, --job-timeout),
# veles/server.py:619-635).
WATCHDOG_STEP_S = 60.0
WATCHDOG_INIT_S = 300.0


def _watchdog(wf, dp):
    """At N > 1: exit 124 with a [watchdog] line when this rank's step
    makes no progress (decision runs) for VELES_AMD_BENCH_WATCHDOG_S s
    (default 60) after its first step, or reaches no first step within
    VELES_AMD_BENCH_WATCHDOG_INIT_S s (default 300) - a hung collective
    ends the run instead of holding the node."""
    if dp.world_size <= 1:
        return None
    from veles_amd.parallel.faults import Watchdog
    timeout = float(os.environ.get("VELES_AMD_BENCH_WATCHDOG_S",
                                   WATCHDOG_STEP_S))
    init = float(os.environ.get("VELES_AMD_BENCH_WATCHDOG_INIT_S",
                                WATCHDOG_INIT_S))
    wd = None

    def expire():
        print("[watchdog] bench.py rank %d: no training step finished for "
              "%.0f s%s (a collective waiting on a peer?); exiting 124" %
              (dp.rank, wd._limit(), "" if wd.armed else
               " before the first step"), file=sys.stderr, flush=True)
        os._exit(124)
    wd = Watchdog(timeout, on_expire=expire, init_timeout=init)
    return wd.install(wf)


def _stall_for_test(dp):
    """VELES_AMD_BENCH_STALL_RANK=r (tests only): rank r stops making
    progress after the warmup, as a rank stuck in a collective would."""
    r = os.environ.get("VELES_AMD_BENCH_STALL_RANK")
    if r is not None and int(r) == dp.rank and dp.world_size > 1:
        while True:
            time.sleep(1.0)


def _graph_warmup(warmup):
    from veles_amd.utils.config import root, get
    ra = os.environ.get("VELES_AMD_LOADER_RUNAHEAD", "1" if get(
        root.common.engine.loader_runahead, False) else "0") != "0"
    per = warmup // 2 if ra else warmup
    return max(0, min(2, per - 1))


def dp_report(dp, store, backend, wf=None):
    """What the multi-rank step did, for reading an N > 1 result
    (docs/PARALLEL.md): ranks seen by the process group, RCCL version,
    gradient bucket layout and wire dtype, and the compute stream's exposed
    wait for the collectives (max over ranks)."""
    import torch
    if not dp.multi:
        return {"grad_allreduce": "none (one rank: no collectives)"}
    import torch.distributed as dist
    info = {"world_size_seen": dist.get_world_size(), "backend": dp.backend,
            "solo": bool(dp.solo)}
    if dp.backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            info["rccl_version"] = ".".join(str(x) for x in v) \
                if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001
            info["rccl_version"] = "unknown (%s)" % e
    rep = None
    if store is not None:
        lay = store.bucket_layout()
        info["buckets_mb"] = [mb for mb, _ in lay]
        info["grad_dtype"] = store.grad_dtype
        info["overlapped_update"] = bool(store._overlap_update())
        info["graph_backward"] = bool(store.graph_safe())
        info["graph_backward_mode"] = store.graph_backward_mode()
        segs = {sg.name: sg for sg in getattr(wf, "graph_segments_", [])} \
            if wf is not None else {}
        bw = segs.get("backward")
        if bw is not None and bw.validations:
            # each key's first captured pass against the eager pass
            # (models/params.py CaptureValidator): True = kept
            info["capture_validated"] = list(bw.validations)
        rep = store.comm_report()
        tl = store.timeline_report()
        if tl is not None:
            info["bucket_timeline"] = tl
    info["per_rank_graphs"] = _per_rank_graphs(dp, store, backend, wf)
    ms = torch.tensor([rep["mean_ms"] if rep else -1.0], dtype=torch.float64)
    if dp.world_size > 1:
        if backend == "hip":
            ms = ms.cuda()
        dp.all_reduce_max(ms)
    v = float(ms.cpu()[0])
    info["exposed_allreduce_ms_per_step"] = round(v, 4) if v >= 0 else None
    info["stats_from"] = "untimed eager steps after the timed region"
    info["grad_allreduce"] = "bucketed %s all-reduce (%s, %d buckets), " \
        "launched per bucket during backward" % (
            "RCCL" if dp.backend == "nccl" else dp.backend,
            info.get("grad_dtype", "float32"), len(info.get("buckets_mb", [])))
    return info


def _per_rank_graphs(dp, store, backend, wf):
    """[rank, graph_backward, forward captures, forward replays, backward
    captures, backward replays] of every rank (all-gathered)."""
    import torch
    import torch.distributed as dist
    segs = {s.name: s for s in getattr(wf, "graph_segments_", [])} \
        if wf is not None else {}
    row = [dp.rank, int(bool(store.graph_safe())) if store else 0]
    for name in ("forward", "backward"):
        s = segs.get(name)
        row += [s.captures, s.replays] if s is not None else [0, 0]
    t = torch.tensor(row, dtype=torch.int64)
    if backend == "hip":
        t = t.cuda()
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[int(v) for v in o.cpu()] for o in out]


if __name__ == "__main__":
    sys.exit(main())
