"""Ensemble loader: the member models' test outputs as features
(reference veles/loader/ensemble.py:53-159).

Reads the JSON written by ``--ensemble-test`` (veles_amd/ensemble/
manager.py): ``models[i]["Output"]`` is [n_samples, n_out] for member i.
The feature vector of a sample is the concatenation of all members' outputs
([n_models, n_out] per sample).  Members with a permuted label mapping are
remapped to the first member's order.  In training mode the true labels
come from ``labels`` (a list) or ``labels_file`` (.npy).
"""
from __future__ import annotations

import json

import numpy

from veles_amd.loader.base import TEST, TRAIN
from veles_amd.loader.fullbatch import FullBatchLoader

__all__ = ["EnsembleLoader"]


class EnsembleLoader(FullBatchLoader):
    MAPPING = "ensemble"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("normalization_type", "none")
        super().__init__(workflow, **kwargs)
        self.file = kwargs["file"]
        self.labels = kwargs.get("labels")
        self.labels_file = kwargs.get("labels_file")

    def load_data(self):
        with open(self.file) as f:
            ens = json.load(f)
        outs, ref = [], None
        for m in ens["models"]:
            o = numpy.asarray(m.get("Output"), dtype=numpy.float32)
            if o.ndim != 2:
                raise ValueError("model %s has no test Output" % m.get("id"))
            lbls = m.get("Labels") or list(range(o.shape[1]))
            if ref is None:
                ref = lbls
            elif lbls != ref:
                if sorted(map(str, lbls)) != sorted(map(str, ref)):
                    raise ValueError("model %s has a different label set" %
                                     m.get("id"))
                pos = {str(v): i for i, v in enumerate(ref)}
                o2 = numpy.zeros_like(o)
                for j, v in enumerate(lbls):
                    o2[:, pos[str(v)]] = o[:, j]
                o = o2
            if outs and o.shape != outs[0].shape:
                raise ValueError("model %s output shape %s != %s" % (
                    m.get("id"), o.shape, outs[0].shape))
            outs.append(o)
        data = numpy.stack(outs, axis=1)  # [n, models, out]
        n = len(data)
        self.class_lengths = [0, 0, 0]
        if self.testing:
            self.class_lengths[TEST] = n
        else:
            self.class_lengths[TRAIN] = n
            lab = self.labels
            if lab is None and self.labels_file:
                lab = numpy.load(self.labels_file, allow_pickle=False)
            if lab is None:
                raise ValueError("EnsembleLoader needs labels / labels_file "
                                 "to train")
            lab = numpy.asarray(lab)
            names = list(ref)
            self.labels_mapping = {v: i for i, v in enumerate(names)}
            self.reversed_labels_mapping = names
            self.original_labels = numpy.array(
                [self.labels_mapping.get(v, v) for v in lab.tolist()],
                numpy.int32)
        self.original_data.reset(numpy.ascontiguousarray(data))
