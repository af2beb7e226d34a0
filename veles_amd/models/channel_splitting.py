"""Channel splitter / merger (Znicz ``channel_splitting``,
docs/source/manualrst_veles_workflow_parameters.rst:476,485).

``ChannelSplitter`` turns an NHWC minibatch [N, H, W, C] into N*C
single-channel images [N*C, H, W] (channel-major within a sample), so that
per-channel sub-networks can run as one batched GEMM; ``ChannelMerger``
is its inverse ([N*C, H, W] -> [N, H, W, C], needs ``n_channels``).  The
reference's exact layout is not recoverable (Znicz sources are absent), so
this contract is pinned in tests/test_znicz_extra.py ("parity unpinned").
Both are one permute-copy on the device; the backward units apply the
inverse permutation to the error.
"""
from __future__ import annotations

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase

__all__ = ["ChannelSplitter", "ChannelMerger", "GDChannelSplitter",
           "GDChannelMerger"]


def _split(x):
    N, H, W, C = x.shape
    return x.permute(0, 3, 1, 2).reshape(N * C, H, W)


def _merge(x, C):
    NC, H, W = x.shape[:3]
    return x.reshape(NC // C, C, H, W).permute(0, 2, 3, 1)


class _Reshaper(AcceleratedUnit):
    hide_from_registry = True
    has_weights = False

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.output = Array(shallow_pickle=True)
        self.demand("input")

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        self.run()

    def run(self):
        self.output.devmem = self.transform(self.input.devmem).contiguous()


class ChannelSplitter(_Reshaper):
    MAPPING = "channel_splitter"

    def initialize(self, device=None, **kwargs):
        shape = tuple(self.input.shape)
        if len(shape) != 4:
            raise ValueError("%s needs NHWC input, got %s" % (self, shape))
        self.n_channels = shape[3]
        super().initialize(device=device, **kwargs)

    def transform(self, x):
        return _split(x)


class ChannelMerger(_Reshaper):
    MAPPING = "channel_merger"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.n_channels = int(kwargs["n_channels"])

    def transform(self, x):
        if x.dim() == 4 and x.shape[3] == 1:
            x = x.squeeze(-1)
        return _merge(x, self.n_channels)


class GDChannelSplitter(GradientDescentBase):
    MAPPING = "channel_splitter"

    def run(self):
        if not self.need_err_input:
            return
        C = self.input.devmem.shape[3]
        self.err_input.devmem = _merge(self.err_output.devmem, C).contiguous()


class GDChannelMerger(GradientDescentBase):
    MAPPING = "channel_merger"

    def run(self):
        if not self.need_err_input:
            return
        err = _split(self.err_output.devmem)
        self.err_input.devmem = err.reshape(self.input.devmem.shape) \
            .contiguous()
