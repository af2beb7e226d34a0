"""CIFAR-style pickled batches (reference veles/loader/pickles.py:55-215,
``PicklesImageFullBatchLoader``).

Each file is a pickled dict with ``data`` ([N, C*H*W] uint8, channel-planar)
and ``labels`` (or ``fine_labels``).  Only the user's own dataset files are
read this way (pickle executes code: never point it at untrusted files).
Images are converted to NHWC uint8 and served from the device.
"""
from __future__ import annotations

import pickle

import numpy

from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.fullbatch import FullBatchLoader

__all__ = ["PicklesImageFullBatchLoader"]


class PicklesImageFullBatchLoader(FullBatchLoader):
    MAPPING = "full_batch_pickles_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.paths = {TEST: list(kwargs.get("test_pickles", ())),
                      VALID: list(kwargs.get("validation_pickles", ())),
                      TRAIN: list(kwargs.get("train_pickles", ()))}
        self.image_shape = tuple(kwargs.get("shape", (32, 32, 3)))

    @staticmethod
    def _read(path):
        with open(path, "rb") as f:
            d = pickle.load(f, encoding="bytes")
        get = (lambda k: d.get(k) if k in d else d.get(k.encode()))
        data = numpy.asarray(get("data"), dtype=numpy.uint8)
        labels = get("labels")
        if labels is None:
            labels = get("fine_labels")
        return data, numpy.asarray(labels, dtype=numpy.int32)

    def load_data(self):
        H, W, C = self.image_shape
        datas, labels = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            for p in self.paths[cls]:
                d, l = self._read(p)
                d = d.reshape(-1, C, H, W).transpose(0, 2, 3, 1)
                datas.append(d)
                labels.append(l)
                self.class_lengths[cls] += len(d)
        self.original_data.reset(numpy.ascontiguousarray(
            numpy.concatenate(datas)))
        lab = numpy.concatenate(labels)
        names = sorted(set(lab.tolist()))
        self.labels_mapping = {v: i for i, v in enumerate(names)}
        self.reversed_labels_mapping = names
        self.original_labels = numpy.array(
            [self.labels_mapping[v] for v in lab.tolist()], numpy.int32)
        self._apply_validation_ratio()
