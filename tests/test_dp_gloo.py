"""Synchronous data parallelism on the CPU (gloo, world_size 2): two ranks
training on halves of each global minibatch end with weights identical to
each other and to a single process training on the whole global batch."""
import os
import socket

import numpy
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(rank, world, port, out, steps, layers_name, bucket_mb=None,
           overlap="1", backend="cpu", grad_dtype="float32"):
    import torch
    os.environ["VELES_AMD_DP_GRAD_DTYPE"] = grad_dtype
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    os.environ["VELES_AMD_DP_OVERLAP_UPDATE"] = overlap
    torch.set_num_threads(1)
    from veles_amd.utils.config import root
    if bucket_mb is not None:
        root.common.engine.dp.bucket_mb = bucket_mb
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models import zoo
    from veles_amd.parallel.dp import DataParallel
    import veles_amd.loader  # noqa: F401
    dp = DataParallel(backend="gloo") if world > 1 else None
    la = DummyLauncher()
    if dp is not None:
        la.dp_ = dp
    wf = StandardWorkflow(
        la, loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 100, 400),
                       "minibatch_size": 40,
                       "normalization_type": "mean_disp"},
        layers=getattr(zoo, layers_name)(),
        decision_config={"max_epochs": None, "fail_iterations": None})
    wf.initialize(device=Device(backend=backend))
    wf.run_steps(steps)
    if backend != "cpu":
        torch.cuda.synchronize()
    w = [f.weights_master.cpu().numpy().copy() for f in wf.forwards
         if getattr(f, "_pw_", None) is not None]
    numpy.savez(out % rank, *w)
    if dp is not None:
        st = wf.param_store_
        # small buckets: several per-bucket updates on the overlap path
        assert bucket_mb is None or len(st.buckets) >= 2, len(st.buckets)
        assert st._overlap == (overlap != "0")
        assert st.grad_dtype == grad_dtype
        dp.shutdown()


@pytest.mark.parametrize("layers_name,bucket_mb,overlap", [
    ("mnist_fc", None, "1"), ("lenet", None, "1"), ("lenet", 0.05, "1"),
    ("mnist_fc", 0.02, "0")])
def test_dp_matches_single_process(tmp_path, layers_name, bucket_mb,
                                   overlap):
    """Per-bucket updates (overlapped with the backward on a GPU side
    stream) and the single fused update give the same weights."""
    steps = 6
    out = str(tmp_path / "w%d.npz")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_train, args=(r, 2, port, out, steps,
                                               layers_name, bucket_mb,
                                               overlap))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    single = str(tmp_path / "s%d.npz")
    p = ctx.Process(target=_train, args=(0, 1, port, single, steps,
                                         layers_name))
    p.start()
    p.join(240)
    assert p.exitcode == 0
    w0 = numpy.load(out % 0)
    w1 = numpy.load(out % 1)
    ws = numpy.load(single % 0)
    for k in w0.files:
        numpy.testing.assert_array_equal(w0[k], w1[k])
        numpy.testing.assert_allclose(w0[k], ws[k], rtol=1e-4, atol=1e-5)


# ------------------------------------------- benchmark-topology equivalence
def _small_alexnet_dropout():
    """The reduced AlexNet of tests/test_e2e_gpu.py (grouped convolutions,
    LRN -> max pooling, conv1 with stride 4: the space-to-depth gather on the
    GPU) with dropout after the fully-connected layer."""
    from test_e2e_gpu import _small_alexnet
    layers = _small_alexnet()
    layers.insert(-1, {"type": "dropout", "->": {"dropout_ratio": 0.5}})
    return layers


def _fp8_net():
    g = {"learning_rate": 0.05, "gradient_moment": 0.9}
    return [
        {"type": "conv_str", "->": {"n_kernels": 16, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "conv_str", "->": {"n_kernels": 32, "kx": 3, "ky": 3,
                                    "padding": 1}, "<-": dict(g)},
        {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
        {"type": "all2all_str", "->": {"output_sample_shape": 64},
         "<-": dict(g)},
        {"type": "softmax", "->": {"output_sample_shape": 10}, "<-": dict(g)}]


def _conv_image_net():
    g = {"learning_rate": 0.05, "gradient_moment": 0.9}
    return [{"type": "conv_relu", "->": {"n_kernels": 8, "kx": 3, "ky": 3},
             "<-": dict(g)},
            {"type": "max_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
            {"type": "softmax", "->": {"output_sample_shape": 2},
             "<-": dict(g)}]


_NETS = {"small_alexnet_dropout": _small_alexnet_dropout,
         "fp8_net": _fp8_net, "conv_image_net": _conv_image_net}


def _train_spec(rank, world, port, out, steps, spec, backend="cpu"):
    """One rank (or the single process, world 1) of a topology described by
    ``spec``: {"loader", "config", "net", "precision"}; saves the weights
    and the rank's last minibatch indices."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from veles_amd.utils.config import root
    root.common.engine.precision_type = spec.get("precision", "float32")
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.parallel.dp import DataParallel
    from veles_amd.prng import random_generator
    import veles_amd.loader  # noqa: F401
    random_generator.get().seed(5)
    dp = DataParallel(backend="gloo") if world > 1 else None
    la = DummyLauncher()
    if dp is not None:
        la.dp_ = dp
    wf = StandardWorkflow(
        la, loader_name=spec["loader"], loader_config=dict(spec["config"]),
        layers=_NETS[spec["net"]](),
        decision_config={"max_epochs": None, "fail_iterations": None})
    wf.initialize(device=Device(backend=backend))
    wf.run_steps(steps)
    if backend != "cpu":
        torch.cuda.synchronize()
    w = [f.weights_master.float().cpu().numpy().copy() for f in wf.forwards
         if getattr(f, "_pw_", None) is not None]
    numpy.savez(out % rank, *w)
    if dp is not None:
        dp.shutdown()


def _equivalence(tmp_path, spec, steps, rtol, atol, backend="cpu"):
    """2 ranks x (B / 2) against 1 process x B: both ranks bit-identical,
    and within (rtol, atol) of the single process."""
    out = str(tmp_path / "w%d.npz")
    single = str(tmp_path / "s%d.npz")
    ctx = mp.get_context("spawn")
    for world, dst in ((2, out), (1, single)):
        port = _free_port()
        procs = [ctx.Process(target=_train_spec,
                             args=(r, world, port, dst, steps, spec,
                                   backend))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(400)
            assert p.exitcode == 0
    w0, w1, ws = (numpy.load(out % 0), numpy.load(out % 1),
                  numpy.load(single % 0))
    worst = 0.0
    for k in w0.files:
        numpy.testing.assert_array_equal(w0[k], w1[k])
        numpy.testing.assert_allclose(w0[k], ws[k], rtol=rtol, atol=atol)
        worst = max(worst, float(numpy.abs(w0[k] - ws[k]).max()))
    return worst


def test_dp_reduced_alexnet_matches_single_process(tmp_path):
    """Grouped convolutions, LRN -> pooling and seeded dropout at 2 ranks:
    the dropout masks are drawn at the rank's global element offset, so
    the ranks draw exactly the single process's masks."""
    spec = {"loader": "synthetic_images", "net": "small_alexnet_dropout",
            "config": {"dataset": "imagenet", "n_classes": 16,
                       "class_lengths": (0, 0, 64), "minibatch_size": 8,
                       "normalization_type": "mean_disp", "seed": 9}}
    _equivalence(tmp_path, spec, 3, 1e-4, 1e-6)


def test_dp_fp8_workflow_matches_single_process(tmp_path):
    """float8 delayed scaling at 2 ranks: the per-step amaxes are reduced
    with MAX over the ranks before they enter the history
    (engine.dp.fp8_amax_sync), so both ranks scale with the global batch's
    amax, as one process does; what remains is the fp32 sum order of the
    two shards' gradients."""
    spec = {"loader": "synthetic_images", "net": "fp8_net",
            "precision": "float8",
            "config": {"dataset": "mnist", "class_lengths": (0, 0, 400),
                       "minibatch_size": 50, "normalization_type":
                       "mean_disp", "seed": 7, "noise": 110.0}}
    _equivalence(tmp_path, spec, 4, 1e-3, 1e-5)


def _png_tree(root, per=8):
    from PIL import Image
    rs = numpy.random.RandomState(0)
    for ci, c in enumerate(("cat", "dog")):
        d = os.path.join(root, c)
        os.makedirs(d, exist_ok=True)
        for i in range(per):
            a = (rs.rand(10, 12, 3) * 60 + ci * 150).astype(numpy.uint8)
            Image.fromarray(a).save(os.path.join(d, "%s_%d.png" % (c, i)))
    return root


def test_dp_streaming_image_loader_sharded(tmp_path):
    """The streaming FileImageLoader under rank sharding: each rank decodes
    its half of every global minibatch (prefetching the next one), random
    crops and mirrors are drawn for the whole global minibatch and sliced,
    and the trained weights equal one process's over the global batch."""
    root = _png_tree(str(tmp_path / "img"))
    spec = {"loader": "file_image", "net": "conv_image_net",
            "config": {"train_paths": [root], "size": (12, 10),
                       "crop": (8, 8), "mirror": "random",
                       "minibatch_size": 8, "decode_workers": 2,
                       "normalization_type": "mean_disp"}}
    _equivalence(tmp_path, spec, 5, 1e-4, 1e-6)


@pytest.mark.gpu
def test_dp_reduced_alexnet_on_gpu(tmp_path):
    """The same topology through the HIP kernels (2 ranks on one GPU, gloo
    collectives): grouped implicit-GEMM convolutions, the fused LRN ->
    pooling, conv1's space-to-depth gather and the device dropout at the
    rank offset; both ranks agree bit for bit and stay within split-K
    atomic noise of one process over the global batch."""
    spec = {"loader": "synthetic_images", "net": "small_alexnet_dropout",
            "precision": "bfloat16",
            "config": {"dataset": "imagenet", "n_classes": 16,
                       "class_lengths": (0, 0, 128), "minibatch_size": 16,
                       "normalization_type": "mean_disp", "seed": 9,
                       "generate_on_device": False}}
    worst = _equivalence(tmp_path, spec, 3, 2e-2, 2e-3, backend="hip")
    print("reduced AlexNet 2 ranks vs 1: max weight difference %g" % worst)


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_dp_bf16_gradient_buckets(tmp_path, overlap):
    """engine.dp.grad_dtype = bfloat16: each bucket goes over the wire as a
    bf16 shadow and is cast back into the fp32 gradient before the fp32
    master update.  Both ranks agree bit for bit and stay within bf16
    rounding of the fp32-wire single-process run."""
    steps = 6
    out = str(tmp_path / "w%d.npz")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_train, args=(r, 2, port, out, steps,
                                               "lenet", 0.05, overlap,
                                               "cpu", "bfloat16"))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    single = str(tmp_path / "s%d.npz")
    p = ctx.Process(target=_train, args=(0, 1, port, single, steps, "lenet"))
    p.start()
    p.join(240)
    assert p.exitcode == 0
    w0, w1, ws = (numpy.load(out % 0), numpy.load(out % 1),
                  numpy.load(single % 0))
    differs = False
    for k in w0.files:
        numpy.testing.assert_array_equal(w0[k], w1[k])
        numpy.testing.assert_allclose(w0[k], ws[k], rtol=2e-2, atol=2e-3)
        differs |= not numpy.array_equal(w0[k], ws[k])
    assert differs, "bf16 wire gave bit-identical weights: not in effect"


def _run_ranks(world, out, steps, layers_name, bucket_mb, overlap, backend):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_train, args=(r, world, port, out, steps,
                                               layers_name, bucket_mb,
                                               overlap, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0


@pytest.mark.gpu
def test_dp_overlapped_update_on_gpu(tmp_path):
    """Two ranks on the GPU (gloo carries the collectives; RCCL refuses two
    ranks on one device): the per-bucket updates on the side stream, which
    wait on each bucket's all-reduce while the backward continues, end with
    the same weights as the single fused update after the backward, and
    both ranks agree bit for bit."""
    steps = 5
    ov = str(tmp_path / "ov%d.npz")
    fu = str(tmp_path / "fu%d.npz")
    _run_ranks(2, ov, steps, "lenet", 0.05, "force", "hip")
    _run_ranks(2, fu, steps, "lenet", 0.05, "0", "hip")
    a0, a1, b0 = (numpy.load(ov % 0), numpy.load(ov % 1), numpy.load(fu % 0))
    for k in a0.files:
        assert numpy.isfinite(a0[k]).all()
        numpy.testing.assert_array_equal(a0[k], a1[k])
        # split-K f32 atomics make runs differ in the last bits; a stale
        # or raced bucket update would differ by a whole update (~1e-3)
        numpy.testing.assert_allclose(a0[k], b0[k], rtol=1e-4, atol=1e-6)


def _train_local(steps, monkeypatch, acc):
    import torch
    if acc > 1:
        monkeypatch.setenv("VELES_AMD_DP_ACCUMULATE", str(acc))
    else:
        monkeypatch.delenv("VELES_AMD_DP_ACCUMULATE", raising=False)
    torch.set_num_threads(1)
    from veles_amd.prng import random_generator
    for i in range(4):
        random_generator.get(i).seed(1234 + i)
    numpy.random.seed(1234)
    torch.manual_seed(1234)
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow, zoo
    import veles_amd.loader  # noqa: F401
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 0, 400),
                       "minibatch_size": 40,
                       "normalization_type": "mean_disp"},
        layers=zoo.mnist_fc(),
        decision_config={"max_epochs": None, "fail_iterations": None})
    wf.initialize(device=Device(backend="cpu"))
    assert wf.loader.max_minibatch_size == 40 // acc
    wf.run_steps(steps * acc)
    return [f.weights_master.numpy().copy() for f in wf.forwards
            if getattr(f, "_pw_", None) is not None]


def test_gradient_accumulation_keeps_global_batch(monkeypatch):
    """acc micro-steps of B/acc samples == one step of B samples: the
    elastic-shrink path (parallel/launch.py ``shrink``) keeps the global
    batch this way."""
    ref = _train_local(3, monkeypatch, 1)
    got = _train_local(3, monkeypatch, 2)
    for a, b in zip(ref, got):
        numpy.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


def test_spawn_ranks_shrinks_after_failure(tmp_path):
    """A rank that fails once is dropped on respawn; survivors accumulate
    world0 / world1 micro-steps."""
    import sys
    from veles_amd.parallel.launch import spawn_ranks
    script = tmp_path / "r.py"
    script.write_text(
        "import os, sys\n"
        "w = int(os.environ['WORLD_SIZE']); r = int(os.environ['RANK'])\n"
        "if w == 3 and r == 1: sys.exit(7)\n"
        "open(os.path.join(%r, 'r%%d_w%%d' %% (r, w)), 'w').write(\n"
        "    os.environ.get('VELES_AMD_DP_ACCUMULATE', '1') + ' ' +\n"
        "    os.environ['VELES_AMD_DEVICE'])\n" % str(tmp_path))
    rc = spawn_ranks("0-2", [sys.executable, str(script)], respawn=1,
                     snapshot_dir=str(tmp_path), poll=0.05, shrink=True)
    assert rc == 0
    assert (tmp_path / "r0_w2").read_text() == "2 0"
    assert (tmp_path / "r1_w2").read_text() == "2 2"


def test_watchdog_kicked_by_decision_and_expires():
    """--job-timeout: the decision unit's run kicks the watchdog; a stall
    longer than the timeout fires on_expire (os._exit(124) by default)."""
    import threading
    import time
    from veles_amd.parallel.faults import Watchdog

    class Dec(object):
        def run(self):
            pass

    class Wf(object):
        decision = Dec()

    fired = threading.Event()
    wd = Watchdog(0.4, on_expire=fired.set).install(Wf)
    for _ in range(6):
        Wf.decision.run()
        time.sleep(0.1)
    assert not fired.is_set()
    assert fired.wait(3.0)
    wd.stop()


def test_spawn_ranks_multi_node_rank_layout(tmp_path):
    """Two "nodes" of two ranks each on one host: global ranks 0-3 meet at
    one rendezvous and each rank sees its node-local rank and device."""
    import sys
    import threading
    from veles_amd.parallel.launch import spawn_ranks
    script = tmp_path / "r.py"
    script.write_text(
        "import os\n"
        "import torch.distributed as dist\n"
        "import torch\n"
        "dist.init_process_group('gloo')\n"
        "t = torch.tensor([float(dist.get_rank())])\n"
        "dist.all_reduce(t)\n"
        "e = os.environ\n"
        "open(os.path.join(%r, 'r' + e['RANK']), 'w').write(' '.join(\n"
        "    [e['LOCAL_RANK'], e['WORLD_SIZE'], e['GROUP_RANK'],\n"
        "     e['VELES_AMD_DEVICE'], str(int(t.item()))]))\n"
        "dist.destroy_process_group()\n" % str(tmp_path))
    port = _free_port()
    rcs = [None, None]

    def node(r):
        rcs[r] = spawn_ranks("0,1", [sys.executable, str(script)],
                             poll=0.05, nnodes=2, node_rank=r,
                             master_addr="127.0.0.1", master_port=port)
    ts = [threading.Thread(target=node, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert rcs == [0, 0]
    for g in range(4):
        assert (tmp_path / ("r%d" % g)).read_text() == "%d 4 %d %d 6" % (
            g % 2, g // 2, g % 2)


def test_multi_node_launch_validation_and_argv():
    from veles_amd.__main__ import _strip_launch_flags
    from veles_amd.parallel.launch import spawn_ranks
    with pytest.raises(ValueError):
        spawn_ranks("0", ["true"], nnodes=2, node_rank=0)
    with pytest.raises(ValueError):
        spawn_ranks("0", ["true"], nnodes=2, node_rank=2,
                    master_addr="127.0.0.1", master_port=1)
    with pytest.raises(ValueError):
        spawn_ranks("0", ["true"], nnodes=2, node_rank=0, shrink=True,
                    master_addr="127.0.0.1", master_port=1)
    argv = ["wf.py", "-", "--gpus", "0-7", "--nnodes=2", "--node-rank", "1",
            "--master-addr", "10.0.0.1", "--master-port=29500", "root.x=1"]
    assert _strip_launch_flags(argv) == ["wf.py", "-", "root.x=1"]


def _train_snap(rank, world, port, snapdir, steps):
    import torch
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from veles_amd.backends import Device
    from veles_amd.dummy import DummyLauncher
    from veles_amd.models import StandardWorkflow
    from veles_amd.models import zoo
    from veles_amd.parallel.dp import DataParallel
    from veles_amd.utils.config import root
    import veles_amd.loader  # noqa: F401
    root.common.disable.snapshotting = False
    dp = DataParallel(backend="gloo", timeout_s=60)
    la = DummyLauncher()
    la.dp_ = dp
    # the clocks of the two ranks disagree as much as they can: rank 0
    # always finds the interval elapsed, rank 1 never does.  The decision
    # must still be collective (rank 0's), or rank 0 waits in the export
    # barrier while rank 1 enters the next gradient all-reduce.
    wf = StandardWorkflow(
        la, loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 40, 80),
                       "minibatch_size": 40,
                       "normalization_type": "mean_disp"},
        layers=zoo.mnist_fc(),
        decision_config={"max_epochs": None, "fail_iterations": None},
        snapshotter_config={"prefix": "dp", "directory": snapdir,
                            "interval": 1, "compression": "",
                            "time_interval": 0.0 if rank == 0 else 1e9})
    wf.initialize(device=Device(backend="cpu"))
    wf.run_steps(steps)
    dp.barrier()
    dp.shutdown()


def test_dp_snapshotter_decision_is_collective(tmp_path):
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_train_snap,
                         args=(r, 2, port, str(tmp_path), 6))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert codes == [0, 0]
    snaps = [f for f in os.listdir(tmp_path) if f.startswith("dp_") and
             "current" not in f]
    assert snaps, "rank 0 wrote no snapshot"


def test_multi_node_respawn_needs_shared_snapshot_dir(tmp_path, monkeypatch):
    """Only global rank 0 writes snapshots; a node whose snapshot directory
    is not shared with the others would resume stale state."""
    import threading
    from veles_amd.parallel.launch import check_shared_dir, spawn_ranks
    monkeypatch.setenv("VELES_AMD_SHARED_DIR_TIMEOUT", "0.5")
    # node 1 alone: node 0's marker never shows up -> refused before launch
    with pytest.raises(ValueError, match="shared"):
        spawn_ranks("0", ["true"], respawn=1, nnodes=2, node_rank=1,
                    master_addr="127.0.0.1", master_port=1,
                    snapshot_dir=str(tmp_path / "private"))
    # both nodes see one directory: accepted
    shared = str(tmp_path / "shared")
    ok = [None, None]

    def node(r):
        ok[r] = check_shared_dir(shared, 2, r, "job", timeout=10)
    ts = [threading.Thread(target=node, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(20)
    assert ok == [True, True]
    # what that job left under the tag proves nothing to the next launch:
    # node 1 alone (node 0 not started) must still time out, and so must
    # node 0 alone
    for r in (1, 0):
        with pytest.raises(ValueError, match="shared"):
            check_shared_dir(shared, 2, r, "job", timeout=0.6)
    # and a fresh pair under the same tag passes again
    ok = [None, None]
    ts = [threading.Thread(target=node, args=(r,)) for r in (1, 0)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(20)
    assert ok == [True, True]


def _digest_rank(rank, port, path, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2",
                       "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    from veles_amd.launcher import Launcher
    la = Launcher(backend="cpu", snapshot_file=path % rank)
    try:
        la.initialize()
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, "mismatch" if "different snapshots" in str(e)
               else str(e)))
    la.dp_.shutdown()


def test_ranks_must_resume_the_same_snapshot(tmp_path):
    ctx = mp.get_context("spawn")
    for same in (True, False):
        for r in (0, 1):
            (tmp_path / ("s%d" % r)).write_bytes(
                b"snap" + (b"" if same else bytes([r])))
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_digest_rank,
                          args=(r, port, str(tmp_path / "s%d"), q))
              for r in (0, 1)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
        res = dict(q.get(timeout=5) for _ in ps)
        assert set(res.values()) == {"ok" if same else "mismatch"}
