"""Avatar: a double-buffered clone of another unit's outputs so that the
producer (usually the loader) can run ahead (reference veles/avatar.py:21-129).

MI355X form: ``run()`` copies the source tensors device-to-device on the
copy-stream and records an event the consumers' compute stream waits on;
the compute stream never stalls on the host."""
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
