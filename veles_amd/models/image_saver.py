"""ImageSaver: writes the input images of the current minibatch to disk as
PNG files, by class (test / validation / train), with the true and the
predicted label in the file name.

Znicz' ``ImageSaver`` (linked by ``StandardWorkflow.link_image_saver``,
docs/source/manualrst_veles_workflow_creation.rst:454-470; the Znicz source
is absent) dumps the misclassified samples of the epoch that improved the
validation error so a user can look at what the network gets wrong.  Here:

* softmax networks: samples whose argmax differs from the label are saved
  (``only_errors=False`` saves every sample);
* MSE networks (``target`` linked): the input, the output and the target
  side by side;
* at most ``limit`` images per class pass; a class directory is emptied
  when a new pass over that class starts (``clear_dirs``), detected from the
  loader's ``minibatch_offset`` going back;
* rank 0 only, host copies of one minibatch only - never on the hot path
  (the builder gates it with ``~decision.improved``).
"""
from __future__ import annotations

import os

import numpy

from veles_amd.loader.base import CLASS_NAME
from veles_amd.units import Unit

__all__ = ["ImageSaver", "to_uint8_image"]


def _host(v, n=None):
    if v is None:
        return None
    t = getattr(v, "devmem", None)
    if t is not None:
        a = t.detach().float().cpu().numpy()
    elif getattr(v, "mem", None) is not None:
        a = numpy.asarray(v.mem)
    elif hasattr(v, "detach"):
        a = v.detach().float().cpu().numpy()
    else:
        a = numpy.asarray(v)
    return a if n is None else a[:n]


def to_uint8_image(a):
    """Min-max scale one sample to a uint8 HxW or HxWx3 image (other channel
    counts show channel 0)."""
    a = numpy.asarray(a, dtype=numpy.float64)
    if a.ndim == 1:
        side = int(numpy.ceil(numpy.sqrt(a.size)))
        b = numpy.zeros(side * side)
        b[:a.size] = a
        a = b.reshape(side, side)
    if a.ndim == 3 and a.shape[-1] not in (1, 3):
        a = a[..., 0]
    if a.ndim == 3 and a.shape[-1] == 1:
        a = a[..., 0]
    lo, hi = float(a.min()), float(a.max())
    return numpy.clip((a - lo) / (hi - lo + 1e-12) * 255.0, 0,
                      255).astype(numpy.uint8)


class ImageSaver(Unit):
    MAPPING = "image_saver"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.out_dir = kwargs.get("out_dir", os.path.join(
            kwargs.get("directory", "."), "image_saver"))
        self.limit = int(kwargs.get("limit", 100))
        self.only_errors = kwargs.get("only_errors", True)
        self.clear_dirs = kwargs.get("clear_dirs", True)
        self.sample_shape = kwargs.get("sample_shape")
        self.target = None
        self.labels = None
        self.indices = None
        self.demand("input", "output", "minibatch_class", "minibatch_size",
                    "minibatch_offset")
        self.saved = [0, 0, 0]
        self.files = []

    def init_unpickled(self):
        super().init_unpickled()
        self.last_offset_ = [None, None, None]

    @property
    def disabled(self):
        launcher = getattr(self.workflow, "workflow", None)
        return getattr(launcher, "rank", 0) not in (0, None)

    def class_dir(self, cls):
        return os.path.join(self.out_dir, CLASS_NAME[cls])

    def _start_pass(self, cls):
        off = int(self.minibatch_offset)
        last = self.last_offset_[cls]
        self.last_offset_[cls] = off
        if last is not None and off > last:
            return
        self.saved[cls] = 0
        d = self.class_dir(cls)
        os.makedirs(d, exist_ok=True)
        if self.clear_dirs:
            for f in os.listdir(d):
                if f.endswith(".png"):
                    os.remove(os.path.join(d, f))

    def run(self):
        if self.disabled:
            return
        cls = int(self.minibatch_class)
        self._start_pass(cls)
        room = self.limit - self.saved[cls]
        if room <= 0:
            return
        n = int(self.minibatch_size)
        x = _host(self.input, n)
        y = _host(self.output, n)
        if self.sample_shape is not None:
            x = x.reshape((n,) + tuple(self.sample_shape))
        lab = _host(self.labels, n)
        idx = _host(self.indices, n)
        tgt = _host(self.target, n)
        from PIL import Image
        for i in range(n):
            if room <= 0:
                break
            num = int(idx[i]) if idx is not None else i
            if tgt is None:
                pred = int(numpy.argmax(y[i].reshape(-1)))
                true = int(lab[i]) if lab is not None else -1
                if self.only_errors and pred == true:
                    continue
                img = to_uint8_image(x[i])
                name = "%d_as_%d.%d.png" % (true, pred, num)
            else:
                parts = [to_uint8_image(a.reshape(x[i].shape)
                                        if a.size == x[i].size else a)
                         for a in (x[i], y[i], tgt[i])]
                h = max(p.shape[0] for p in parts)
                parts = [numpy.pad(p, ((0, h - p.shape[0]),) +
                                   ((0, 0),) * (p.ndim - 1)) for p in parts]
                if len({p.ndim for p in parts}) > 1:
                    parts = [p if p.ndim == 2 else p.mean(-1).astype(
                        numpy.uint8) for p in parts]
                img = numpy.concatenate(parts, axis=1)
                err = float(numpy.sqrt(numpy.mean(
                    (y[i].reshape(-1) - tgt[i].reshape(-1)) ** 2)))
                name = "%.6f.%d.png" % (err, num)
            fn = os.path.join(self.class_dir(cls), name)
            Image.fromarray(img).save(fn)
            self.files.append(fn)
            self.saved[cls] += 1
            room -= 1
