"""ZeroFiller (Znicz ``weights_zerofilling.ZeroFiller``,
docs/source/manualrst_veles_workflow_parameters.rst:499).

Keeps the weights of the preceding layer block-diagonal: with ``grouping``
g, input features and output neurons are split into g groups and every
weight connecting different groups is reset to zero after each update
(grouped fully connected / conv layers emulated through a mask).  In the
data path the unit is the identity.  On the device it is one multiply of
the layer's master weights by a cached 0/1 mask (and the bf16 copy), hooked
into the parameter store right after each fused update.
"""
from __future__ import annotations

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase

__all__ = ["ZeroFiller", "GDZeroFiller"]


class ZeroFiller(AcceleratedUnit):
    MAPPING = "zero_filter"
    has_weights = False

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.grouping = int(kwargs.get("grouping", 1))
        self.weights_unit = kwargs.get("weights_unit")
        self.output = Array(shallow_pickle=True)
        self.demand("input")

    def init_unpickled(self):
        super().init_unpickled()
        self.mask_ = None

    def make_mask(self, shape, like):
        import torch
        out_n = shape[0]
        in_n = 1
        for s in shape[1:]:
            in_n *= s
        g = self.grouping
        if out_n % g or shape[-1] % g:
            raise ValueError("%s: %s not divisible into %d groups" %
                             (self, shape, g))
        rows = torch.arange(out_n, device=like.device) // (out_n // g)
        # group of an input feature = group of its channel (last axis)
        ch = torch.arange(in_n, device=like.device) % shape[-1]
        cols = ch // (shape[-1] // g)
        return (rows[:, None] == cols[None, :]).to(like.dtype).view(shape)

    def apply_mask(self):
        u = self.weights_unit
        if u is None or self.grouping <= 1:
            return
        w = u.weights_master
        if self.mask_ is None or self.mask_.shape != w.shape:
            self.mask_ = self.make_mask(tuple(w.shape), w)
        w.mul_(self.mask_)
        lp = u.weights_lp
        if lp is not w:
            lp.copy_(w)

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        self.output.devmem = self.input.devmem
        u = self.weights_unit
        if u is not None and getattr(u, "store_", None) is not None:
            hooks = u.store_.post_update_hooks
            hooks[:] = [h for h in hooks
                        if getattr(h, "__self__", None) is not self]
            hooks.append(self.apply_mask)
        self.apply_mask()

    def run(self):
        # the mask is re-applied by the store after every update
        self.output.devmem = self.input.devmem


class GDZeroFiller(GradientDescentBase):
    MAPPING = "zero_filter"

    def run(self):
        self.err_input.devmem = self.err_output.devmem
