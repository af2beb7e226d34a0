"""Fan-out branches of the Python engine on HIP streams (units._Branches,
SURVEY §2.6 "intra-process graph concurrency"; reference veles/units.py:
485-505): with engine.parallel_fanout on a GPU workflow, the two branches of
an InputJoiner diamond run on two different streams forked from the compute
stream, the join waits for both, and the output equals the serial run's -
eagerly and inside a captured HIP graph."""
import pytest
import torch

from veles_amd import ops
from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.backends import Device
from veles_amd.dummy import DummyWorkflow
from veles_amd.input_joiner import InputJoiner
from veles_amd.memory import Array
from veles_amd.units import TrivialUnit, _Scheduler
from veles_amd.utils.config import root

pytestmark = pytest.mark.gpu


class _Branch(AcceleratedUnit):
    """out = x @ w (a few GEMMs long, so the branches overlap)"""

    def __init__(self, workflow, x, w, reps=4, **kw):
        super().__init__(workflow, **kw)
        self.x, self.w, self.reps = x, w, reps
        self.output = Array(shallow_pickle=True)
        self.stream_seen = None

    def initialize(self, device=None, **kw):
        super().initialize(device=device, **kw)
        self.output.devmem = torch.empty(self.x.shape[0], self.w.shape[1],
                                         dtype=torch.bfloat16,
                                         device=self.x.device)

    def run(self):
        self.stream_seen = torch.cuda.current_stream().cuda_stream
        y = self.x
        for _ in range(self.reps):
            y = ops.gemm(y, self.w, out_dtype=torch.bfloat16)
        self.output.devmem.copy_(y)


def _diamond(dev, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.rand(2048, 2048, generator=g, device="cuda") - 0.5).to(
        torch.bfloat16)
    wa = ((torch.rand(2048, 2048, generator=g, device="cuda") - 0.5) /
          16).to(torch.bfloat16)
    wb = ((torch.rand(2048, 2048, generator=g, device="cuda") - 0.5) /
          16).to(torch.bfloat16)
    wf = DummyWorkflow(dev)
    fork = TrivialUnit(wf)
    fork.link_from(wf.start_point)
    a = _Branch(wf, x, wa, name="branch_a")
    b = _Branch(wf, x, wb, name="branch_b")
    a.link_from(fork)
    b.link_from(fork)
    j = InputJoiner(wf, inputs=[a.output, b.output])
    j.link_from(a, b)
    wf.end_point.unlink_from(wf.start_point)
    wf.end_point.link_from(j)
    wf.initialize(device=dev)
    return wf, a, b, j


@pytest.mark.parametrize("graph", [False, True])
def test_diamond_branches_on_streams(graph):
    dev = Device(backend="hip")
    old = root.common.engine.parallel_fanout
    outs = {}
    try:
        for par in (False, True):
            root.common.engine.parallel_fanout = par
            wf, a, b, j = _diamond(dev, 3)
            if graph:
                # capture one pass on a side stream, replay it
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                wf.run()          # warm-up (allocations, library state)
                torch.cuda.synchronize()
                # the unit graph itself on the capturing stream (wf.run()
                # would switch to the device's compute stream); the
                # finished pass left every unit stopped
                for u in wf:
                    u.stopped = False
                with torch.cuda.stream(s):
                    g.capture_begin()
                    with _Scheduler() as sched:
                        wf.start_point.run_dependent()
                        sched.drain()
                    g.capture_end()
                j.output.devmem.zero_()
                g.replay()
            else:
                wf.run()
            torch.cuda.synchronize()
            outs[par] = j.output.devmem.clone()
            if par:
                base = dev.stream().cuda_stream
                assert a.stream_seen != b.stream_seen
                if not graph:
                    assert base not in (a.stream_seen, b.stream_seen)
                assert j.ran_on_ is not a.ran_on_
            else:
                assert a.stream_seen == b.stream_seen
    finally:
        root.common.engine.parallel_fanout = old
    assert torch.equal(outs[False], outs[True])
    assert float(outs[True].float().abs().sum()) > 0


def test_dead_end_branch_rejoins_for_capture():
    """A branch that never reaches a join (here: the end point links from
    branch a only, b is a dead end) is joined back when the outermost
    scheduler drain ends (_Branches.join_all), so a capture of the pass ends
    cleanly and the replay computes b's output too."""
    dev = Device(backend="hip")
    old = root.common.engine.parallel_fanout
    try:
        root.common.engine.parallel_fanout = True
        g = torch.Generator(device="cuda").manual_seed(5)
        x = (torch.rand(2048, 2048, generator=g, device="cuda") - 0.5).to(
            torch.bfloat16)
        wa = ((torch.rand(2048, 2048, generator=g, device="cuda") - 0.5) /
              16).to(torch.bfloat16)
        wb = ((torch.rand(2048, 2048, generator=g, device="cuda") - 0.5) /
              16).to(torch.bfloat16)
        wf = DummyWorkflow(dev)
        fork = TrivialUnit(wf)
        fork.link_from(wf.start_point)
        a = _Branch(wf, x, wa, name="branch_a")
        b = _Branch(wf, x, wb, name="branch_b")
        a.link_from(fork)
        b.link_from(fork)
        wf.end_point.unlink_from(wf.start_point)
        wf.end_point.link_from(a)
        wf.initialize(device=dev)
        wf.run()
        torch.cuda.synchronize()
        ref = b.output.devmem.clone()
        for u in wf:
            u.stopped = False
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            graph.capture_begin()
            with _Scheduler() as sched:
                wf.start_point.run_dependent()
                sched.drain()
            graph.capture_end()
        b.output.devmem.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert a.stream_seen != b.stream_seen
        assert torch.equal(b.output.devmem, ref)
    finally:
        root.common.engine.parallel_fanout = old
