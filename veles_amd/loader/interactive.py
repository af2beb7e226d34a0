"""Feed-driven loaders for serving: ``InteractiveLoader.feed(sample)`` and
``RestfulLoader.feed(sample, request)``.

Reference: veles/loader/interactive.py:57-216 and loader/restful.py:52-167 —
a one-sample (or few-sample) TEST loader that takes its input from an
external feeder, normalises it with the trained loader's normalizer
(``derive_from``) and blocks until the next input arrives.  Here the queued
samples of one wakeup are batched into one minibatch (up to
``minibatch_size``) so the GEMMs stay MFMA-shaped under load, and the
normalisation runs on the device.  ``feed(None)`` stops the workflow.
"""
from __future__ import annotations

import queue

import numpy

from veles_amd.loader.base import TEST, Loader

__all__ = ["InteractiveLoader", "RestfulLoader"]


class InteractiveLoader(Loader):
    MAPPING = "interactive"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("minibatch_size", 1)
        super().__init__(workflow, **kwargs)
        self._shape = tuple(kwargs["sample_shape"]) \
            if kwargs.get("sample_shape") else None
        self.max_minibatch_size = int(kwargs.get("minibatch_size", 1))
        self.feed_timeout = kwargs.get("feed_timeout", None)
        self.queue_ = queue.Queue()

    def init_unpickled(self):
        super().init_unpickled()
        self.queue_ = queue.Queue()
        self.current_ = []

    @property
    def sample_shape(self):
        return self._shape

    def derive_from(self, loader):
        super().derive_from(loader)
        if self._shape is None:
            self._shape = tuple(loader.sample_shape)

    def load_data(self):
        if self._shape is None:
            raise ValueError("%s: sample_shape is unknown (pass it or "
                             "derive_from a trained loader)" % self)
        self.class_lengths = [self.max_minibatch_size, 0, 0]
        self.has_labels = False

    def create_minibatch_data(self):
        import torch
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        dt = dev.compute_dtype if dev is not None and getattr(
            dev, "is_gpu", False) else torch.float32
        self.minibatch_data.devmem = torch.zeros(
            (self.max_minibatch_size,) + self._shape, dtype=dt, device=tdev)
        self.minibatch_indices.initialize(dev)

    def analyze_dataset(self):
        pass

    def feed(self, sample, context=None):
        """Queue one sample (array-like of ``sample_shape``)."""
        if sample is None:
            self.queue_.put(None)
            return
        a = numpy.asarray(sample, dtype=numpy.float32)
        if a.shape != self._shape:
            a = a.reshape(self._shape)
        self.queue_.put((a, context))

    def _take(self):
        items = [self.queue_.get(timeout=self.feed_timeout)]
        while len(items) < self.max_minibatch_size:
            try:
                items.append(self.queue_.get_nowait())
            except queue.Empty:
                break
        return items

    def run(self):
        import torch
        try:
            items = self._take()
        except queue.Empty:
            items = [None]
        if any(it is None for it in items):
            self.info("feeding stopped")
            wf = self.workflow
            if wf is not None:
                wf.stop()
            return
        n = len(items)
        x = numpy.stack([a for a, _ in items])
        if self.normalizer is not None and \
                self.normalizer.is_initialized:
            self.normalizer.normalize(x.reshape(n, -1))
        t = self.minibatch_data.devmem
        t[:n].copy_(torch.from_numpy(x).to(t.dtype))
        t[n:].zero_()
        self.current_ = [c for _, c in items]
        self.minibatch_class = TEST
        self.minibatch_size = n
        self.global_minibatch_size = n
        self.last_minibatch <<= False
        self.epoch_ended <<= False


class RestfulLoader(InteractiveLoader):
    """Each fed sample carries its HTTP request context; the RESTful API
    unit answers ``current_requests`` after the forward pass."""
    MAPPING = "restful"

    def feed(self, sample, request=None):
        super().feed(sample, request)

    @property
    def current_requests(self):
        return self.current_
