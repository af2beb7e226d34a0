"""Collects the network output over the TEST class in ``--test`` mode.

The reference's ensemble test step reads each member's ``Output`` (the last
layer's activations for every test sample) and ``Labels`` (the label
mapping) from the workflow results (veles/loader/ensemble.py:66-120,
ensemble/test_workflow.py).  Outputs stay on the device until the test
epoch ends; one D2H copy then.
"""
from __future__ import annotations

from veles_amd.loader.base import TEST
from veles_amd.units import Unit
from veles_amd.workflow import IResultProvider

__all__ = ["OutputCollector"]


class OutputCollector(Unit, IResultProvider):
    MAPPING = "output_collector"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "EVALUATOR")
        super().__init__(workflow, **kwargs)
        self.outputs = []
        self.indices = []
        self.demand("output", "minibatch_class", "minibatch_size",
                    "minibatch_indices", "labels_source")

    def init_unpickled(self):
        super().init_unpickled()
        self.chunks_ = []

    def initialize(self, **kwargs):
        self.chunks_ = []
        self.outputs = []
        self.indices = []

    def run(self):
        if self.minibatch_class != TEST:
            return
        n = int(self.minibatch_size)
        out = self.output.devmem
        idx = self.minibatch_indices
        idx = idx.devmem if idx.devmem is not None else idx.mem
        if idx is not None:
            idx = idx[:n].clone() if hasattr(idx, "clone") else \
                idx[:n].copy()
        self.chunks_.append((out[:n].float().clone(), idx))

    def finalize(self):
        import numpy
        outs, ids = [], []
        for o, i in self.chunks_:
            outs.append(o.reshape(o.shape[0], -1).cpu().numpy())
            if i is not None:
                ids.append(numpy.asarray(i.cpu() if hasattr(i, "cpu") else i)
                           .reshape(-1))
        self.chunks_ = []
        if not outs:
            return
        out = numpy.concatenate(outs)
        if ids and sum(len(i) for i in ids) == len(out):
            order = numpy.argsort(numpy.concatenate(ids), kind="stable")
            out = out[order]
        self.outputs = out.tolist()

    def get_metric_names(self):
        return {"Output", "Labels"}

    def get_metric_values(self):
        self.finalize()
        src = self.labels_source
        return {"Output": self.outputs,
                "Labels": list(getattr(src, "reversed_labels_mapping", []))}
