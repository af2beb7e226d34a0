"""HDF5 loaders (reference veles/loader/loader_hdf5.py:48-151).

``h5py`` is not part of this environment; the loader is importable and
fails with a clear message when used without it.  Datasets: ``data`` and
``labels`` per class file (test / validation / train).
"""
from __future__ import annotations

import numpy

from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.fullbatch import FullBatchLoader

__all__ = ["FullBatchHDF5Loader", "HDF5Loader"]


def _h5py():
    try:
        import h5py
    except ImportError:
        raise ImportError("HDF5 loaders need h5py, which is not installed "
                          "(convert the data to .npy and use the numpy "
                          "loader instead)") from None
    return h5py


class FullBatchHDF5Loader(FullBatchLoader):
    MAPPING = "full_batch_hdf5"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.files = {TEST: kwargs.get("test_path"),
                      VALID: kwargs.get("validation_path"),
                      TRAIN: kwargs.get("train_path")}

    def load_data(self):
        h5py = _h5py()
        datas, labels = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            fn = self.files[cls]
            if not fn:
                continue
            with h5py.File(fn, "r") as f:
                datas.append(numpy.asarray(f["data"]))
                labels.append(numpy.asarray(f["labels"]).astype(numpy.int32))
            self.class_lengths[cls] = len(datas[-1])
        self.original_data.reset(numpy.concatenate(datas))
        self.original_labels = numpy.concatenate(labels)
        n = int(self.original_labels.max()) + 1
        self.labels_mapping = {i: i for i in range(n)}
        self.reversed_labels_mapping = list(range(n))


HDF5Loader = FullBatchHDF5Loader
