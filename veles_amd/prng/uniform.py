"""Uniform: device xorshift1024* generator (reference
veles/prng/uniform.py:48-176; kernel ocl/random.cl:42-70).  ``num_states``
states of 16 x uint64; each round produces 16 uint64 per state, interleaved
out[round*16*n + i*n + id]; the numpy model (veles_amd.prng.xorshift1024star)
is bit-exact."""
from __future__ import annotations

import numpy
import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array, roundup
from veles_amd.prng import random_generator
from veles_amd import ops

__all__ = ["Uniform"]


class Uniform(AcceleratedUnit):
    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.num_states = kwargs.get("num_states", 256)
        self.prng = kwargs.get("prng", random_generator.get())
        self.output_bytes = kwargs.get("output_bytes", 0)
        self.states = Array()
        self.output = Array()

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        if not self.states or self.states.size != self.num_states * 16:
            st = self.prng.randint(0, 2 ** 32, self.num_states * 32,
                                   dtype=numpy.uint64).astype(numpy.uint32)
            self.states.reset(st.view(numpy.int64).reshape(
                self.num_states, 16).copy())
        per_round = self.num_states * 16 * 8
        self.output_bytes = roundup(max(self.output_bytes, per_round),
                                    per_round)
        self.states.initialize(self.device)
        self.output.devmem = torch.zeros(self.output_bytes // 8,
                                         dtype=torch.int64,
                                         device=self.torch_device)

    def fill(self, nbytes):
        per_round = self.num_states * 16 * 8
        nbytes = roundup(nbytes, per_round)
        if nbytes > self.output_bytes:
            raise ValueError("nbytes > output_bytes")
        rounds = nbytes // per_round
        out = self.output.devmem[:rounds * self.num_states * 16]
        ops.xorshift1024star(self.states.devmem, rounds, out=out)

    def run(self):
        self.fill(self.output_bytes)
