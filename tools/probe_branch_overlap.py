"""Fan-out branches on HIP streams, traced: an InputJoiner diamond (two
branches of 4 GEMMs 4096^2 each) run with engine.parallel_fanout off, then
on (eager, then a captured HIP graph replay), so that a rocprofv3 kernel
trace shows whether the two branches' kernels overlap in time
(tools/branch_overlap_summary.py reads the trace; VERDICT r3 item 7,
tests/test_branch_streams_gpu.py checks the outputs).

    rocprofv3 --kernel-trace --output-format csv -d OUT -- \\
        python3 tools/probe_branch_overlap.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                ".."))
from veles_amd import ops  # noqa: E402
from veles_amd.accelerated_units import AcceleratedUnit  # noqa: E402
from veles_amd.backends import Device  # noqa: E402
from veles_amd.dummy import DummyWorkflow  # noqa: E402
from veles_amd.input_joiner import InputJoiner  # noqa: E402
from veles_amd.memory import Array  # noqa: E402
from veles_amd.units import TrivialUnit, _Scheduler  # noqa: E402
from veles_amd.utils.config import root  # noqa: E402

S = 4096


class Branch(AcceleratedUnit):
    def __init__(self, workflow, x, w, **kw):
        super().__init__(workflow, **kw)
        self.x, self.w = x, w
        self.output = Array(shallow_pickle=True)

    def initialize(self, device=None, **kw):
        super().initialize(device=device, **kw)
        self.output.devmem = torch.empty(S, S, dtype=torch.bfloat16,
                                         device=self.x.device)

    def run(self):
        y = self.x
        for _ in range(4):
            y = ops.gemm(y, self.w, out_dtype=torch.bfloat16)
        self.output.devmem.copy_(y)


def diamond(dev):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(S, S, generator=g, device="cuda") - 0.5).to(torch.bfloat16)
    wa = ((torch.rand(S, S, generator=g, device="cuda") - 0.5) / 32).to(
        torch.bfloat16)
    wb = ((torch.rand(S, S, generator=g, device="cuda") - 0.5) / 32).to(
        torch.bfloat16)
    wf = DummyWorkflow(dev)
    fork = TrivialUnit(wf)
    fork.link_from(wf.start_point)
    a = Branch(wf, x, wa, name="branch_a")
    b = Branch(wf, x, wb, name="branch_b")
    a.link_from(fork)
    b.link_from(fork)
    j = InputJoiner(wf, inputs=[a.output, b.output])
    j.link_from(a, b)
    wf.end_point.unlink_from(wf.start_point)
    wf.end_point.link_from(j)
    wf.initialize(device=dev)
    return wf


def main():
    dev = Device(backend="hip")
    old = root.common.engine.parallel_fanout
    try:
        for par in (False, True):
            root.common.engine.parallel_fanout = par
            wf = diamond(dev)
            for _ in range(3):
                wf.run()
            torch.cuda.synchronize()
            print("parallel_fanout=%s eager done" % par, flush=True)
        # a captured pass with the fan-out on, replayed
        wf = diamond(dev)
        wf.run()
        torch.cuda.synchronize()
        for u in wf:
            u.stopped = False
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            gr.capture_begin()
            with _Scheduler() as sched:
                wf.start_point.run_dependent()
                sched.drain()
            gr.capture_end()
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        print("graph replay done", flush=True)
    finally:
        root.common.engine.parallel_fanout = old


if __name__ == "__main__":
    main()
