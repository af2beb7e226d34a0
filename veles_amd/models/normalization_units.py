"""Local response normalisation across channels (Znicz ``norm``;
docs/OPS.md §LRN): y_c = x_c * (k + alpha * sum_{|c'-c|<=n/2} x_c'^2)^-beta.
Vectorised over 8 channels of an NHWC pixel (``hvk_lrn_fwd/bwd``).

When a 3x3 max pooling follows (AlexNet norm1/pool1, norm2/pool2) the
StandardWorkflow links them (``fused_into``) and the pooling units run the
fused kernels (``hvk_lrn_pool_fwd/bwd``): the LRN output and the pool
gradient are never materialised, and these units' runs become no-ops."""
from __future__ import annotations

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops

__all__ = ["LRNormalizerForward", "LRNormalizerBackward"]


class _LRNParams(object):
    def _lrn_kwargs(self, kwargs):
        self.alpha = kwargs.get("alpha", 0.0001)
        self.beta = kwargs.get("beta", 0.75)
        self.k = kwargs.get("k", 2.0)
        self.n = int(kwargs.get("n", 5))


class LRNormalizerForward(AcceleratedUnit, _LRNParams):
    MAPPING = "norm"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self._lrn_kwargs(kwargs)
        self.output = Array(shallow_pickle=True)
        self.fused_into = None  # the max pooling unit that computes us
        self.demand("input")

    @property
    def activation(self):
        return 0

    def package_export(self):
        return {"alpha": self.alpha, "beta": self.beta, "k": self.k,
                "n": self.n}

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        import torch
        x = self.input.devmem
        self.output.devmem = torch.zeros(
            tuple(self.input.shape), dtype=x.dtype if x is not None else
            self.compute_dtype, device=self.torch_device)

    @property
    def fused(self):
        p = self.fused_into
        return p is not None and getattr(p, "lrn_fused_active_", False)

    def run(self):
        import torch
        if self.fused:
            return
        x = self.input.devmem
        y = self.output.devmem
        if y is None or y.shape != x.shape or y.dtype != x.dtype or \
                y.device != x.device:
            self.output.devmem = y = torch.empty_like(x)
        ops.lrn_fwd(x, self.n, self.alpha, self.beta, self.k, out=y)


class LRNormalizerBackward(GradientDescentBase, _LRNParams):
    MAPPING = "norm"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._lrn_kwargs(kwargs)

    def run(self):
        fwd = self.forward
        if fwd is not None and getattr(fwd, "fused", False):
            return  # err_input written by the fused pooling backward
        x = self.input.devmem
        ei = self.alloc_err_input(tuple(x.shape))
        aux, aux_act = self.aux_tensor()
        ops.lrn_bwd(x, self.err_output.devmem, self.n, self.alpha, self.beta,
                    self.k, aux=aux, aux_act=aux_act, out=ei)
