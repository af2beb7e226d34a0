"""Minibatch recording and replay (reference veles/loader/saver.py:69-296:
``MinibatchesSaver`` dumps the served minibatches into one compressed file
with an offset table; ``MinibatchesLoader`` random-accesses them).

File layout (own format, little endian)::

    b"VLMB1\\0" | record* | table JSON | u64 table offset | b"VLMB1\\0"

Each record is one minibatch (``numpy.savez`` of data / labels / targets /
indices, trimmed to ``minibatch_size``) compressed with the file's codec
(none / gz / bz2 / xz; snappy is not available here).  The table holds the
codec, sample shape, and per record (offset, length, class, size).  The
loader serves the recorded minibatches as a resident full batch, classes in
recorded order, without reshuffling.
"""
from __future__ import annotations

import bz2
import gzip
import io
import json
import lzma
import struct

import numpy

from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.fullbatch import FullBatchLoader
from veles_amd.units import Unit

__all__ = ["MinibatchesSaver", "MinibatchesLoader", "read_minibatches"]

MAGIC = b"VLMB1\0"
CODECS = {
    "none": (lambda b: b, lambda b: b),
    "gz": (gzip.compress, gzip.decompress),
    "bz2": (bz2.compress, bz2.decompress),
    "xz": (lzma.compress, lzma.decompress),
}


def _to_numpy(arr, n):
    if arr is None:
        return None
    t = getattr(arr, "devmem", None)
    if t is not None:
        return t[:n].float().cpu().numpy() if t.is_floating_point() else \
            t[:n].cpu().numpy()
    m = getattr(arr, "mem", None)
    return None if m is None else numpy.asarray(m[:n])


class MinibatchesSaver(Unit):
    MAPPING = "minibatches_saver"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.file_name = kwargs.get("file_name", "minibatches.dat")
        self.compression = kwargs.get("compression", "gz")
        if self.compression not in CODECS:
            raise ValueError("compression must be one of %s" %
                             sorted(CODECS))
        self.demand("minibatch_data", "minibatch_size", "minibatch_class")
        self.minibatch_labels = None
        self.minibatch_targets = None
        self.minibatch_indices = None

    def init_unpickled(self):
        super().init_unpickled()
        self.file_ = None
        self.table_ = []

    def initialize(self, **kwargs):
        self.file_ = open(self.file_name, "wb")
        self.file_.write(MAGIC)
        self.table_ = []

    def run(self):
        n = int(self.minibatch_size)
        rec = {"data": _to_numpy(self.minibatch_data, n)}
        for k in ("labels", "targets", "indices"):
            v = _to_numpy(getattr(self, "minibatch_" + k), n)
            if v is not None:
                rec[k] = v
        bio = io.BytesIO()
        numpy.savez(bio, **rec)
        blob = CODECS[self.compression][0](bio.getvalue())
        off = self.file_.tell()
        self.file_.write(blob)
        self.table_.append((off, len(blob), int(self.minibatch_class), n))

    def stop(self):
        if self.file_ is None:
            return
        tab = json.dumps({"codec": self.compression,
                          "records": self.table_}).encode()
        off = self.file_.tell()
        self.file_.write(tab)
        self.file_.write(struct.pack("<Q", off))
        self.file_.write(MAGIC)
        self.file_.close()
        self.file_ = None
        self.info("Saved %d minibatches to %s", len(self.table_),
                  self.file_name)


def read_minibatches(path, classes=None):
    """Yield (class, dict of arrays) for every record (in order)."""
    with open(path, "rb") as f:
        if f.read(len(MAGIC)) != MAGIC:
            raise ValueError("%s is not a minibatch file" % path)
        f.seek(-(8 + len(MAGIC)), 2)
        (toff,) = struct.unpack("<Q", f.read(8))
        end = f.tell() - 8
        f.seek(toff)
        table = json.loads(f.read(end - toff))
        dec = CODECS[table["codec"]][1]
        for off, ln, cls, n in table["records"]:
            if classes is not None and cls not in classes:
                continue
            f.seek(off)
            z = numpy.load(io.BytesIO(dec(f.read(ln))), allow_pickle=False)
            yield cls, {k: z[k] for k in z.files}


class MinibatchesLoader(FullBatchLoader):
    MAPPING = "minibatches"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("normalization_type", "none")
        kwargs.setdefault("shuffle_limit", 0)
        super().__init__(workflow, **kwargs)
        self.file_name = kwargs["file_name"]

    def load_data(self):
        per = {TEST: [], VALID: [], TRAIN: []}
        for cls, rec in read_minibatches(self.file_name):
            per[cls].append(rec)
        datas, labels = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            for rec in per[cls]:
                datas.append(rec["data"])
                if "labels" in rec:
                    labels.append(rec["labels"])
                self.class_lengths[cls] += len(rec["data"])
        self.original_data.reset(numpy.concatenate(datas).astype(
            numpy.float32))
        if labels:
            lab = numpy.concatenate(labels).astype(numpy.int32)
            self.original_labels = lab
            n = int(lab.max()) + 1
            self.labels_mapping = {i: i for i in range(n)}
            self.reversed_labels_mapping = list(range(n))
