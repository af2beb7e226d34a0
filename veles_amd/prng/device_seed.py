"""Device-resident seed sequences that survive a snapshot.

Dropout and stochastic pooling keep their per-minibatch seed on the GPU
(``seed_dev_``, advanced by ``hvk_seed_advance`` inside the step, so a
captured HIP graph replays with fresh masks and no host value enters the
kernel arguments).  Transient ``*_`` attributes are not pickled, so without
this module a restored unit re-draws its first seed from its host generator
and the resumed masks differ from those of the uninterrupted run.

The reference saves and restores every generator's state around unit runs
and pickles the whole workflow so that resume is exact
(/root/reference/veles/units.py:859-885, veles/snapshotter.py:387-420;
SURVEY §5.4 "snapshot the HIP RNG state too"): ``save`` reads the current
device seed back into a pickled attribute (``seed_dev_saved``) and ``get``
re-creates the device seed from it on the first run after the restore,
without drawing from the host generator."""
from __future__ import annotations

import torch

__all__ = ["save", "get"]


def save(unit):
    """Copy ``unit.seed_dev_`` to the pickled ``unit.seed_dev_saved``
    (called from ``__getstate__``; the device is synchronised first, so the
    value is that of the last advance issued on any stream)."""
    sd = getattr(unit, "seed_dev_", None)
    if sd is None:
        return
    if sd.is_cuda:
        torch.cuda.synchronize(sd.device)
    unit.seed_dev_saved = int(sd.detach().cpu()[0])


def get(unit, device, draw):
    """The device seed tensor of ``unit`` on ``device``: the live one, the
    one restored from a snapshot, or a fresh one seeded by ``draw()`` (the
    unit's host generator)."""
    sd = getattr(unit, "seed_dev_", None)
    if sd is not None and sd.device == device:
        return sd
    saved = getattr(unit, "seed_dev_saved", None)
    if saved is not None:
        value = int(saved)
        unit.seed_dev_saved = None
    else:
        value = int(draw())
    unit.seed_dev_ = sd = torch.tensor([value], dtype=torch.int32,
                                       device=device)
    return sd
