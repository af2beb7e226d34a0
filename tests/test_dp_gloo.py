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


def _train(rank, world, port, out, steps, layers_name):
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
    wf.initialize(device=Device(backend="cpu"))
    wf.run_steps(steps)
    w = [f.weights_master.numpy().copy() for f in wf.forwards
         if getattr(f, "_pw_", None) is not None]
    numpy.savez(out % rank, *w)
    if dp is not None:
        dp.shutdown()


@pytest.mark.parametrize("layers_name", ["mnist_fc", "lenet"])
def test_dp_matches_single_process(tmp_path, layers_name):
    steps = 6
    out = str(tmp_path / "w%d.npz")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_train, args=(r, 2, port, out, steps,
                                               layers_name))
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
    a, b, s = (numpy.load(f % 0 if "s" not in f.split("/")[-1][:1] else f % 0)
               for f in (out, out.replace("%d", "1").replace(".npz", "") +
                         "%d.npz" if False else out, single))
    w0 = numpy.load(out % 0)
    w1 = numpy.load(out % 1)
    ws = numpy.load(single % 0)
    for k in w0.files:
        numpy.testing.assert_array_equal(w0[k], w1[k])
        numpy.testing.assert_allclose(w0[k], ws[k], rtol=1e-4, atol=1e-5)
