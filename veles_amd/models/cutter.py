"""Cutter: crop a window out of NHWC images, and its backward (Znicz
``cutter.Cutter`` / ``cutter.GDCutter``,
docs/source/manualrst_veles_workflow_parameters.rst:490).

``padding`` = (left, top, right, bottom) is what is cut away.  Forward is a
strided device copy; the backward scatters err_output into a zeroed
err_input of the input's shape.
"""
from __future__ import annotations

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.conv import norm_padding
from veles_amd.models.nn_units import GradientDescentBase

__all__ = ["Cutter", "GDCutter"]


class Cutter(AcceleratedUnit):
    MAPPING = "cutter"
    has_weights = False

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.padding = norm_padding(kwargs.get("padding"))
        self.output = Array(shallow_pickle=True)
        self.demand("input")

    def window(self, shape):
        l, t, r, b = self.padding
        H, W = shape[1], shape[2]
        if t + b >= H or l + r >= W:
            raise ValueError("%s: cut %s leaves nothing of %s" %
                             (self, self.padding, shape))
        return slice(t, H - b), slice(l, W - r)

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        import torch
        x = self.input.devmem
        ys, xs = self.window(tuple(x.shape))
        shape = (x.shape[0], ys.stop - ys.start, xs.stop - xs.start) + \
            tuple(x.shape[3:])
        self.output.devmem = torch.zeros(shape, dtype=x.dtype,
                                         device=x.device)

    def run(self):
        x = self.input.devmem
        ys, xs = self.window(tuple(x.shape))
        self.output.devmem.copy_(x[:, ys, xs])


class GDCutter(GradientDescentBase):
    MAPPING = "cutter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.padding = norm_padding(kwargs.get("padding"))

    def run(self):
        fwd = self.forward
        x = self.input.devmem
        ei = self.alloc_err_input(tuple(x.shape), dtype=x.dtype)
        ei.zero_()
        ys, xs = (fwd.window(tuple(x.shape)) if fwd is not None else
                  Cutter.window(self, tuple(x.shape)))
        ei[:, ys, xs] = self.err_output.devmem.to(ei.dtype)
