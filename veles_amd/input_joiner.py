"""InputJoiner: feature-wise concatenation of N minibatch inputs into
[batch, sum sample_size] (reference veles/input_joiner.py:48-212; dynamic
``input_i`` / ``offset_i`` / ``length_i`` attributes, ``link_inputs``)."""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd import ops

__all__ = ["InputJoiner"]


class InputJoiner(AcceleratedUnit):
    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.output = Array(shallow_pickle=True)
        self.num_inputs = kwargs.get("num_inputs", 0)
        inputs = kwargs.get("inputs")
        if inputs:
            self.link_inputs(*inputs)

    def link_inputs(self, *pairs):
        """pairs: Arrays, or (unit, attr) tuples."""
        for i, p in enumerate(pairs):
            name = "input_%d" % (self.num_inputs + i)
            if isinstance(p, tuple):
                self.link_attrs(p[0], (name, p[1]))
            else:
                setattr(self, name, p)
        self.num_inputs += len(pairs)

    @property
    def inputs(self):
        return [getattr(self, "input_%d" % i) for i in range(self.num_inputs)]

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        ins = self.inputs
        if not ins:
            raise AttributeError("InputJoiner has no inputs")
        b = ins[0].shape[0]
        off = 0
        for i, a in enumerate(ins):
            n = a.size // a.shape[0]
            setattr(self, "offset_%d" % i, off)
            setattr(self, "length_%d" % i, n)
            off += n
        dt = ins[0].devmem.dtype if ins[0].devmem is not None else \
            torch.float32
        self.output.devmem = torch.zeros(b, off, dtype=dt,
                                         device=self.torch_device)

    def run(self):
        ops.join([a.devmem for a in self.inputs], out=self.output.devmem)
