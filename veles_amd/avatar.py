"""Avatar: a double-buffered clone of another unit's outputs so that the
producer (usually the loader) can run ahead (reference veles/avatar.py:21-129).

MI355X form: ``run()`` copies the source tensors device-to-device on the
copy-stream and records an event the consumers' compute stream waits on;
the compute stream never stalls on the host.

What this does not do: let the producer's NEXT device fill run beside the
current step's compute.  The full-batch loaders fill on the compute stream
(one fused gather kernel: 0.18 ms of AlexNet's 7.35 ms b1024 step), and a
real run-ahead would alternate two buffers - which a HIP-graph-captured
forward cannot follow (it replays the pointers it captured) without one
graph per buffer parity - while a single-buffer clone adds a copy of the
whole minibatch (320 MB for the space-to-depth AlexNet input) to save the
fill it hides.  Host-side run-ahead lives in the streaming image loaders
(``loader/image.py``: threaded decode, pinned staging, side-stream copy,
next-minibatch prefetch)."""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array

__all__ = ["Avatar"]


class Avatar(AcceleratedUnit):
    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "LOADER")
        super().__init__(workflow, **kwargs)
        self.reals = {}
        self._remembers_gates = False

    def init_unpickled(self):
        super().init_unpickled()
        self.copy_stream_ = None

    def clone(self, unit, *attrs):
        for a in attrs:
            src = getattr(unit, a)
            if isinstance(src, Array):
                dst = Array(shallow_pickle=True)
                setattr(self, a, dst)
                self.reals[a] = (unit, a)
            else:
                self.link_attrs(unit, a)
        return self

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        for a, (unit, name) in self.reals.items():
            src = getattr(unit, name).devmem
            if src is not None:
                getattr(self, a).devmem = torch.empty_like(src)
        if self.is_gpu:
            self.copy_stream_ = torch.cuda.Stream(self.device.index)

    def run(self):
        if self.copy_stream_ is not None:
            cur = torch.cuda.current_stream()
            self.copy_stream_.wait_stream(cur)
            with torch.cuda.stream(self.copy_stream_):
                for a, (unit, name) in self.reals.items():
                    getattr(self, a).devmem.copy_(getattr(unit, name).devmem,
                                                  non_blocking=True)
            cur.wait_stream(self.copy_stream_)
        else:
            for a, (unit, name) in self.reals.items():
                getattr(self, a).devmem.copy_(getattr(unit, name).devmem)
