"""Pooling layers and their backward units (Znicz ``pooling`` /
``gd_pooling``; docs/OPS.md §Pooling).

NHWC, window ``kx`` x ``ky``, ``sliding`` (x, y) (defaults to the window);
windows start inside the input and the last one may be partial (ceil).
max / avg / maxabs run as ``hvk_pool_fwd`` (8 channels per lane) with the
argmax offset kept for the backward GATHER (``hvk_pool_bwd``, deterministic,
no atomics).  Stochastic variants draw the window element with probability
proportional to its (absolute) value during training and use the weighted
average at test time (``hvk_stochastic_pool``, counter-based uniforms from a
device-resident seed).  Depooling scatters through the same gather kernel
(``hvk_pool_bwd``) and its backward is ``hvk_gather``.
"""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase
from veles_amd.prng import device_seed, random_generator
from veles_amd import ops

__all__ = ["Pooling", "MaxPooling", "AvgPooling", "MaxAbsPooling",
           "StochasticPooling", "StochasticAbsPooling",
           "StochasticPoolingDepooling", "StochasticAbsPoolingDepooling",
           "GDPooling", "GDMaxPooling", "GDAvgPooling", "GDMaxAbsPooling",
           "Depooling"]


class Pooling(AcceleratedUnit):
    hide_from_registry = True
    MODE = "max"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.kx = int(kwargs.get("kx", 2))
        self.ky = int(kwargs.get("ky", 2))
        s = kwargs.get("sliding", (self.kx, self.ky))
        self.sliding = (s, s) if isinstance(s, int) else tuple(s)
        self.output = Array(shallow_pickle=True)
        self.input_offset = Array(shallow_pickle=True)
        self.fused_lrn = None  # LRN unit computed by this pooling (fused)
        # input_offset read by another unit (depooling): keep it in the flat
        # int32 format
        self.offsets_exported = False
        self.demand("input")

    def init_unpickled(self):
        super().init_unpickled()
        self.lrn_fused_active_ = False
        self.argmax_free_ = False

    @property
    def activation(self):
        return 0

    def _in(self):
        x = self.input.devmem
        return x.unsqueeze(-1) if x.dim() == 3 else x

    def package_export(self):
        return {"kx": self.kx, "ky": self.ky, "sliding": list(self.sliding)}

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        shape = tuple(self.input.shape)
        if len(shape) == 3:
            shape = shape + (1,)
        B, H, W, C = shape
        OH, OW = ops.pool_out_size(H, W, self.ky, self.kx, self.sliding[1],
                                   self.sliding[0])
        dt = self.input.devmem.dtype if self.input.devmem is not None \
            else self.compute_dtype
        self.output.devmem = torch.zeros(B, OH, OW, C, dtype=dt,
                                         device=self.torch_device)
        lrn = self.fused_lrn
        # non-overlapping 2 x 2 windows on the GPU: no argmax tensor at all,
        # the GD unit recomputes the choice from the input (ops.pool2_bwd)
        self.argmax_free_ = self.is_gpu and lrn is None and \
            not self.offsets_exported and \
            type(self) in (MaxPooling, AvgPooling, MaxAbsPooling) and \
            ops.pool2_ok(shape, self.ky, self.kx, self.sliding)
        if not self.argmax_free_:
            self.input_offset.devmem = torch.zeros(B, OH, OW, C,
                                                   dtype=torch.int32,
                                                   device=self.torch_device)
        self.lrn_fused_active_ = lrn is not None and self.MODE == "max" and \
            len(tuple(self.input.shape)) == 4 and \
            ops.lrn_pool_fusable(C, lrn.n, self.ky, self.kx, self.sliding)
        if self.lrn_fused_active_ and self.is_gpu and \
                tuple(self.sliding) == (2, 2) and not self.offsets_exported:
            # the fused pair keeps its argmax private: one byte per element
            # (window-local index) instead of an int32 offset
            self.input_offset.devmem = torch.zeros(
                B, OH, OW, C, dtype=torch.uint8, device=self.torch_device)

    def run(self):
        if self.lrn_fused_active_:
            lrn = self.fused_lrn
            ops.lrn_pool_fwd(lrn.input.devmem, lrn.n, lrn.alpha, lrn.beta,
                             lrn.k, self.ky, self.kx, self.sliding,
                             out=self.output.devmem,
                             argmax=self.input_offset.devmem)
            return
        x = self._in()
        if self.argmax_free_:
            from veles_amd.models.conv import (fp8_input_consumer,
                                               fp8_input_target)
            y = self.output.devmem
            q8, qs = fp8_input_target(self, y) if y is not None and \
                y.is_cuda else (None, None)
            ops.pool2_fwd(x, self.MODE, out=y, q8=q8, q8_scaler=qs)
            if q8 is not None:
                fp8_input_consumer(self).x8_fresh_ = True
            return
        B, H, W, C = x.shape
        OH, OW = ops.pool_out_size(H, W, self.ky, self.kx, self.sliding[1],
                                   self.sliding[0])
        y = self.output.devmem
        if y is None or tuple(y.shape) != (B, OH, OW, C) or y.dtype != x.dtype \
                or y.device != x.device:
            self.output.devmem = y = torch.zeros(B, OH, OW, C, dtype=x.dtype,
                                                 device=x.device)
            if self.MODE != "avg":
                self.input_offset.devmem = torch.zeros(
                    B, OH, OW, C, dtype=torch.int32, device=x.device)
        ops.pool_fwd(x, self.ky, self.kx, self.sliding, self.MODE, out=y,
                     argmax=self.input_offset.devmem
                     if self.MODE != "avg" else None)


class MaxPooling(Pooling):
    MAPPING = "max_pooling"
    MODE = "max"


class AvgPooling(Pooling):
    MAPPING = "avg_pooling"
    MODE = "avg"


class MaxAbsPooling(Pooling):
    MAPPING = "maxabs_pooling"
    MODE = "maxabs"


class StochasticPooling(Pooling):
    """Training: sample a window element with p ~ max(x, 0) (or |x|);
    testing: probability-weighted average.  ``input_offset`` records the
    sampled element for the max-style backward."""
    MAPPING = "stochastic_pooling"
    MODE = "max"
    USE_ABS = False

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.rand = kwargs.get("rand", random_generator.get())
        self.uniform_seed = 0

    def init_unpickled(self):
        super().init_unpickled()
        self.seed_dev_ = None

    def _draw_seed(self):
        self.uniform_seed = int(self.rand.randint(0, 2 ** 31 - 1))
        return self.uniform_seed

    def __getstate__(self):
        device_seed.save(self)   # exact resume of the device draws
        return super().__getstate__()

    def run(self):
        x = self._in()
        B, H, W, C = x.shape
        OH, OW = ops.pool_out_size(H, W, self.ky, self.kx, self.sliding[1],
                                   self.sliding[0])
        y = self.output.devmem
        if y is None or tuple(y.shape) != (B, OH, OW, C) or \
                y.dtype != x.dtype or y.device != x.device:
            self.output.devmem = y = torch.zeros(B, OH, OW, C, dtype=x.dtype,
                                                 device=x.device)
        off = self.input_offset.devmem
        if off is None or tuple(off.shape) != (B, OH, OW, C) or \
                off.dtype != torch.int32 or off.device != x.device:
            self.input_offset.devmem = off = torch.zeros(
                B, OH, OW, C, dtype=torch.int32, device=x.device)
        train = not bool(getattr(self.workflow, "testing", False))
        if x.is_cuda:
            # device-resident seed sequence (graph-safe, like dropout)
            # (restored from a snapshot: device_seed.get)
            sd = device_seed.get(self, x.device, self._draw_seed)
            if train:
                ops.seed_advance(sd)
            ops.stochastic_pool(x, self.ky, self.kx, self.sliding,
                                self.USE_ABS, train, seed_dev=sd, out=y,
                                argmax=off)
            return
        if train:
            self.uniform_seed = int(self.rand.randint(0, 2 ** 31 - 1))
        ops.stochastic_pool(x, self.ky, self.kx, self.sliding, self.USE_ABS,
                            train, seed=self.uniform_seed, out=y, argmax=off)


class StochasticAbsPooling(StochasticPooling):
    MAPPING = "stochastic_abs_pooling"
    USE_ABS = True


class StochasticPoolingDepooling(StochasticPooling):
    """Pool then scatter back to the input geometry (output has the input
    shape, zeros except at the sampled positions)."""
    MAPPING = "stochastic_pool_depool"

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        self.pooled_ = None

    def run(self):
        # pool into a private buffer, then scatter the drawn values back to
        # the input geometry (the pooling backward's gather kernel)
        x = self._in()
        out = self.output.devmem
        if out is None or tuple(out.shape) != tuple(x.shape) or \
                out.dtype != x.dtype or out.device != x.device:
            out = torch.zeros(x.shape, dtype=x.dtype, device=x.device)
        self.output.devmem = self.pooled_
        super().run()
        self.pooled_ = self.output.devmem
        ops.pool_bwd(self.pooled_, self.input_offset.devmem, tuple(x.shape),
                     self.ky, self.kx, self.sliding, "max", out=out)
        self.output.devmem = out


class StochasticAbsPoolingDepooling(StochasticPoolingDepooling):
    MAPPING = "stochastic_abs_pool_depool"
    USE_ABS = True


class Depooling(AcceleratedUnit):
    """Inverse of a max pooling: scatter ``input`` to the positions recorded
    in ``get_output_shape_from.input_offset`` (Znicz depooling)."""
    MAPPING = "depooling"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.output = Array(shallow_pickle=True)
        self.demand("input", "input_offset", "output_shape_source")

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        src = self.output_shape_source
        x = self.input.devmem
        self.output.devmem = torch.zeros(tuple(src.shape), dtype=x.dtype,
                                         device=x.device)

    def run(self):
        # a scatter-add of x to the recorded offsets IS the max-pooling
        # backward's gather (hvk_pool_bwd, no atomics) given the pooling's
        # window geometry; without it, a device scatter
        x = self.input.devmem
        src = self.output_shape_source.devmem
        out = self.output.devmem
        if out is None or tuple(out.shape) != tuple(src.shape) or \
                out.dtype != x.dtype:
            out = torch.zeros(tuple(src.shape), dtype=x.dtype,
                              device=x.device)
        geo = getattr(self, "geometry", None)
        shape4 = tuple(src.shape) if src.dim() == 4 else \
            tuple(src.shape) + (1,)
        if geo is not None:
            ky, kx, sliding = geo
            ops.pool_bwd(x.reshape(x.shape[0], x.shape[1], x.shape[2], -1),
                         self.input_offset.devmem, shape4, ky, kx, sliding,
                         "max", out=out.view(shape4))
        else:
            flat = torch.zeros(src.numel(), dtype=x.dtype, device=x.device)
            flat.index_put_((self.input_offset.devmem.reshape(-1).long(),),
                            x.reshape(-1), accumulate=True)
            out.copy_(flat.view(src.shape))
        self.output.devmem = out


class GDDepooling(GradientDescentBase):
    """Backward of Depooling: gather err_output at the recorded offsets."""
    MAPPING = "depooling"

    def run(self):
        if not self.need_err_input:
            return
        fwd = self.forward
        off = fwd.input_offset.devmem
        ei = self.alloc_err_input(tuple(self.input.devmem.shape),
                                  self.err_output.devmem.dtype)
        ops.gather(self.err_output.devmem, off, out=ei.view(off.shape))


class GDPoolDepool(GradientDescentBase):
    """Backward of the stochastic pool-depool units: the output keeps the
    input geometry, so err passes through at the sampled positions only."""
    MAPPING = "stochastic_pool_depool"

    def run(self):
        if not self.need_err_input:
            return
        fwd = self.forward
        err = self.err_output.devmem
        off = fwd.input_offset.devmem
        # err passes at the drawn positions: gather there, scatter back
        g = ops.gather(err, off)
        ei = self.alloc_err_input(tuple(err.shape), err.dtype)
        ops.pool_bwd(g, off, tuple(err.shape) if err.dim() == 4 else
                     tuple(err.shape) + (1,), fwd.ky, fwd.kx, fwd.sliding,
                     "max", out=ei.view(tuple(err.shape) if err.dim() == 4
                                        else tuple(err.shape) + (1,)))


class GDPooling(GradientDescentBase):
    hide_from_registry = True
    MODE = "max"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.kx = int(kwargs.get("kx", 2))
        self.ky = int(kwargs.get("ky", 2))
        s = kwargs.get("sliding", (self.kx, self.ky))
        self.sliding = (s, s) if isinstance(s, int) else tuple(s)
        self.fused_lrn_gd = None  # GD unit of a fused LRN below
        self.demand("input_offset")

    def run(self):
        err = self.err_output.devmem
        fwd = self.forward
        if fwd is not None and getattr(fwd, "lrn_fused_active_", False):
            # LRN -> pool fused backward straight into the LRN GD unit's
            # err_input (its own run is a no-op)
            lrn, lgd = fwd.fused_lrn, self.fused_lrn_gd
            x = lrn.input.devmem
            ei = lgd.alloc_err_input(tuple(x.shape))
            aux, aux_act = lgd.aux_tensor()
            ops.lrn_pool_bwd(x, err, self.input_offset.devmem, lrn.n,
                             lrn.alpha, lrn.beta, lrn.k, self.ky, self.kx,
                             self.sliding, aux=aux, aux_act=aux_act, out=ei)
            return
        x = self.input.devmem
        shape = tuple(x.shape) if x.dim() == 4 else tuple(x.shape) + (1,)
        ei = self.alloc_err_input(shape)
        aux, aux_act = self.aux_tensor()
        if fwd is not None and getattr(fwd, "argmax_free_", False):
            from veles_amd.models.gd_conv import (fp8_grad_consumer,
                                                  fp8_grad_target)
            q8, qs = fp8_grad_target(self, ei) if ei.is_cuda else (None, None)
            ops.pool2_bwd(x, err, self.MODE, aux=aux, aux_act=aux_act, out=ei,
                          q8=q8, q8_scaler=qs)
            if q8 is not None:
                fp8_grad_consumer(self).dy8_fresh_ = True
            return
        if aux is not None and aux.dim() == 3:
            aux = aux.unsqueeze(-1)
        ops.pool_bwd(err, self.input_offset.devmem
                     if self.MODE != "avg" else None, shape, self.ky, self.kx,
                     self.sliding, self.MODE, aux=aux, aux_act=aux_act, out=ei)
        if x.dim() == 3:
            self.err_input.devmem = ei.squeeze(-1)


class GDMaxPooling(GDPooling):
    MAPPING = "max_pooling"
    MODE = "max"


class GDAvgPooling(GDPooling):
    MAPPING = "avg_pooling"
    MODE = "avg"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.undemand("input_offset")
        self.input_offset = None


class GDMaxAbsPooling(GDPooling):
    MAPPING = "maxabs_pooling"
    MODE = "maxabs"
