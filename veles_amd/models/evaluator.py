"""Evaluators: loss gradient + error accounting (Znicz ``evaluator``;
docs/source/manualrst_veles_workflow_parameters.rst:143-166).

EvaluatorSoftmax: one fused kernel per minibatch (``hvk_softmax_ce``):
softmax, err_output = (p - onehot) / global_batch, argmax error count, CE
loss, optional confusion matrix.  Metrics accumulate ON THE DEVICE per
minibatch class; the decision unit reads them once per class end, so the
training loop never synchronises the host per step.
EvaluatorMSE: err_output = (y - t) / global_batch, per-sample MSE metrics.
"""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.workflow import IResultProvider
from veles_amd import ops

__all__ = ["EvaluatorSoftmax", "EvaluatorMSE", "EvaluatorBase"]


class EvaluatorBase(AcceleratedUnit, IResultProvider):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "EVALUATOR")
        super().__init__(workflow, **kwargs)
        self.err_output = Array(shallow_pickle=True)
        self.compute_confusion_matrix = kwargs.get(
            "compute_confusion_matrix", False)
        self.mean = kwargs.get("mean", True)
        self.demand("output", "batch_size", "global_batch_size",
                    "minibatch_class")

    def init_unpickled(self):
        super().init_unpickled()
        self.metrics_ = None

    def ensure_metrics(self, n=3):
        m = self.metrics_
        if m is None or m.device != self.torch_device:
            self.metrics_ = torch.zeros(3, n, dtype=torch.float32,
                                        device=self.torch_device)
        return self.metrics_

    def take_class_metrics(self, cls):
        """Return the class' accumulated metrics (host numpy) and reset them.
        One small D2H copy; called by the decision at class end."""
        m = self.ensure_metrics()
        v = m[cls].clone()
        m[cls].zero_()
        return v

    def get_metric_names(self):
        return set()

    def get_metric_values(self):
        return {}


class EvaluatorSoftmax(EvaluatorBase):
    MAPPING = "evaluator_softmax"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("labels")
        self.logits = None
        # per class (test / validation / train) [true][predicted] counts of
        # the last finished pass over that class; ``confusion_matrix`` shows
        # the validation one (train when there is no validation set)
        self.confusion_matrix = Array()
        self.confusion_matrixes = [None, None, None]

    def init_unpickled(self):
        super().init_unpickled()
        self.confusion_ = None

    def run(self):
        lg_arr = self.logits if isinstance(self.logits, Array) else None
        if lg_arr is not None and lg_arr.devmem is not None:
            logits = lg_arr.devmem
        else:  # probabilities only: softmax(log p) == p
            logits = torch.log(self.output.devmem.float().clamp(min=1e-30))
        B, C = logits.shape[0], logits.numel() // logits.shape[0]
        err = self.err_output.devmem
        if err is None or tuple(err.shape) != (B, C) or \
                err.device != self.torch_device:
            self.err_output.devmem = err = torch.zeros(
                B, C, dtype=self.compute_dtype, device=self.torch_device)
        m = self.ensure_metrics()
        conf = None
        if self.compute_confusion_matrix:
            if self.confusion_ is None:
                self.confusion_ = torch.zeros(3, C, C, dtype=torch.int32,
                                              device=self.torch_device)
            conf = self.confusion_[self.minibatch_class]
        gb = max(int(self.global_batch_size), 1)
        ops.softmax_ce(logits.reshape(B, C), self.labels.devmem,
                       scale=1.0 / gb if self.mean else 1.0, err=err,
                       metrics=m[self.minibatch_class], confusion=conf)

    def take_confusion(self, cls, shown=True):
        """The confusion counts of class ``cls`` since its last take (summed
        over the data-parallel group); ``shown`` also publishes them as
        ``confusion_matrix``.  Called by the decision at every class end."""
        if self.confusion_ is None:
            return None
        t = self.confusion_[cls]
        from veles_amd.parallel import find_dp
        dp = find_dp(self)
        if dp is not None and dp.world_size > 1:
            dp.all_reduce_sum(t)
        c = t.cpu().numpy().copy()
        t.zero_()
        self.confusion_matrixes[cls] = c
        if shown:
            self.confusion_matrix.reset(c)
        return c


class EvaluatorMSE(EvaluatorBase):
    MAPPING = "evaluator_mse"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("target")
        self.root = kwargs.get("root", True)

    def run(self):
        y = self.output.devmem
        t = self.target.devmem
        B = y.shape[0]
        err = self.err_output.devmem
        if err is None or err.shape != y.shape or err.device != y.device:
            self.err_output.devmem = err = torch.zeros(
                y.shape, dtype=self.compute_dtype, device=self.torch_device)
        m = self.ensure_metrics()
        gb = max(int(self.global_batch_size), 1)
        ops.mse(y, t, scale=1.0 / gb if self.mean else 1.0, err=err,
                metrics=m[self.minibatch_class],
                valid_rows=int(self.batch_size))
