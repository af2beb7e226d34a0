"""Avatar: a double-buffered clone of another unit's outputs so that the
producer (usually the loader) can run ahead (reference veles/avatar.py:21-129).

Every cloned attribute is a SNAPSHOT taken when the avatar runs, as in the
reference's ``clone()`` (veles/avatar.py:38-73):

* Arrays: the device tensors are copied device-to-device on a copy stream;
  an event joins the consumers' compute stream, which never stalls on the
  host;
* mutable host state is copied into the avatar's own object, so consumers
  linked to it keep their identity: lists are refilled, dicts / sets
  cleared and updated, ``Bool`` gates assigned with ``<<=`` (their
  expression links stay intact), numpy arrays copied in place;
* immutable values (numbers, strings, tuples, None) are re-assigned, and
  anything else is deep-copied.

The producer may therefore advance (its minibatch flags, offsets, label
lists) while the consumers still read the avatar's state of the minibatch
they process.

What this does not do: let the producer's NEXT device fill run beside the
current step's compute.  The full-batch loaders fill on the compute stream
(one fused gather kernel: 0.19 ms of AlexNet's 7.2 ms b1024 step), and a
real run-ahead would alternate two buffers - which a HIP-graph-captured
forward cannot follow (it replays the pointers it captured) without one
graph per buffer parity - while a single-buffer clone adds a copy of the
whole minibatch (320 MB for the space-to-depth AlexNet input) to save the
fill it hides.  Host-side run-ahead lives in the streaming image loaders
(``loader/image.py``: threaded decode, pinned staging, side-stream copy,
next-minibatch prefetch)."""
from __future__ import annotations

import copy

import numpy
import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.mutable import Bool

__all__ = ["Avatar"]

_IMMUTABLE = (int, float, complex, str, bytes, bool, type(None), tuple,
              frozenset)


def _snapshot(cur, value):
    """The avatar's copy of ``value``: ``cur`` updated in place where its
    identity matters (consumers may hold it), else a new object."""
    if isinstance(value, _IMMUTABLE):
        return value
    if isinstance(value, Bool) and not isinstance(cur, Bool):
        return Bool(bool(value))   # a plain gate (even of an expression)
    if cur is None or type(cur) is not type(value):
        return copy.deepcopy(value)
    if isinstance(value, list):
        cur[:] = value
    elif isinstance(value, (dict, set)):
        cur.clear()
        cur.update(value)
    elif isinstance(value, Bool):
        cur <<= bool(value)
    elif isinstance(value, numpy.ndarray):
        if cur.shape != value.shape or cur.dtype != value.dtype:
            return value.copy()
        cur[...] = value
    else:
        return copy.deepcopy(value)
    return cur


class Avatar(AcceleratedUnit):
    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "LOADER")
        super().__init__(workflow, **kwargs)
        self.reals = {}    # attribute -> (unit, name) of a device Array
        self.states = {}   # attribute -> (unit, name) of host state
        self._remembers_gates = False

    def init_unpickled(self):
        super().init_unpickled()
        self.copy_stream_ = None

    def clone(self, unit, *attrs):
        for a in attrs:
            src = getattr(unit, a)
            if isinstance(src, Array):
                setattr(self, a, Array(shallow_pickle=True))
                self.reals[a] = (unit, a)
            else:
                setattr(self, a, _snapshot(None, src))
                self.states[a] = (unit, a)
        return self

    def snapshot_states(self):
        """Copy the producer's current host state into the avatar."""
        for a, (unit, name) in self.states.items():
            setattr(self, a, _snapshot(self.__dict__.get(a),
                                       getattr(unit, name)))

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        self.snapshot_states()
        for a, (unit, name) in self.reals.items():
            src = getattr(unit, name).devmem
            if src is not None:
                getattr(self, a).devmem = torch.empty_like(src)
        if self.is_gpu:
            self.copy_stream_ = torch.cuda.Stream(self.device.index)

    def run(self):
        self.snapshot_states()
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
