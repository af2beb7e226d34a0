"""MeanDispNormalizer unit: out = (float(in) - mean) * rdisp per sample
(reference veles/mean_disp_normalizer.py:49-138; numpy model 129-138).
One vectorised ``hvk_mean_disp_normalize`` launch on the GPU."""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd import ops

__all__ = ["MeanDispNormalizer"]


class MeanDispNormalizer(AcceleratedUnit):
    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.output = Array(shallow_pickle=True)
        self.output_dtype = kwargs.get("output_dtype")
        self.demand("input", "mean", "rdisp")

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        for a in (self.input, self.mean, self.rdisp):
            if a.devmem is None or a.devmem.device != self.torch_device:
                a.initialize(self.device)
        dt = self.output_dtype or (torch.float32 if not self.is_gpu
                                   else self.compute_dtype)
        self.output.devmem = torch.zeros(tuple(self.input.shape), dtype=dt,
                                         device=self.torch_device)

    def run(self):
        ops.mean_disp_normalize(self.input.devmem,
                                self.mean.devmem.float().reshape(-1),
                                self.rdisp.devmem.float().reshape(-1),
                                out=self.output.devmem)
