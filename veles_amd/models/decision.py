"""Training-loop decision units (Znicz ``decision``:
docs/source/manualrst_veles_workflow_parameters.rst:601-614).

* sets ``gd_skip`` for non-TRAIN minibatches (GD units are gate-skipped);
* at every class end reads the evaluator's device metrics (all-reduced over
  the data-parallel group so every rank decides identically);
* at epoch end increments ``epoch_number``, tracks the best validation error
  (``improved``), counts ``fail_iterations`` and raises ``complete`` at
  ``max_epochs`` / ``fail_iterations`` / ``max_steps``;
* builds ``snapshot_suffix`` ("validation_1.48_train_0.04" style).
"""
from __future__ import annotations

import time

import numpy

from veles_amd.loader.base import TEST, VALID, TRAIN, CLASS_NAME
from veles_amd.mutable import Bool
from veles_amd.units import Unit
from veles_amd.workflow import IResultProvider

__all__ = ["DecisionBase", "DecisionGD", "DecisionMSE", "TrivialDecision"]


class DecisionBase(Unit, IResultProvider):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "TRAINER")
        super().__init__(workflow, **kwargs)
        self.max_epochs = kwargs.get("max_epochs", None)
        self.fail_iterations = kwargs.get("fail_iterations", 100)
        self.max_steps = kwargs.get("max_steps", None)
        self.complete = Bool(False)
        # step budget (benchmarks): stops the loop at the repeater AFTER the
        # current step's backward, unlike ``complete`` which blocks the GDs
        self.steps_complete = Bool(False)
        self.improved = Bool(False)
        self.train_improved = Bool(False)
        self.gd_skip = Bool(False)
        self.epoch_ended_flag = Bool(False)
        self.snapshot_suffix = ""
        self.train_steps = 0
        self._fails = 0
        self.epoch_timestamps = []
        self.demand("minibatch_class", "last_minibatch", "class_lengths",
                    "epoch_ended", "epoch_number", "minibatch_size")

    def initialize(self, **kwargs):
        self._t0 = time.time()

    def dp_all_reduce(self, vec):
        from veles_amd.parallel import find_dp
        dp = find_dp(self)
        if dp is not None and dp.world_size > 1:
            return dp.all_reduce_sum(vec)
        return vec

    def run(self):
        mc = self.minibatch_class
        self.gd_skip <<= mc != TRAIN
        if mc == TRAIN:
            self.train_steps += 1
        if self.last_minibatch:
            self.on_last_minibatch(mc)
        self.epoch_ended_flag <<= bool(self.epoch_ended)
        if self.epoch_ended:
            self.on_epoch_ended()
        self.steps_complete <<= (self.max_steps is not None and
                                 self.train_steps >= self.max_steps)

    def on_last_minibatch(self, cls):
        pass

    def on_epoch_ended(self):
        pass

    def increment_epoch(self):
        self.epoch_number = self.epoch_number + 1
        self.epoch_timestamps.append(time.time())
        if self.max_epochs is not None and \
                self.epoch_number >= self.max_epochs:
            self.complete <<= True


class TrivialDecision(DecisionBase):
    MAPPING = "trivial"

    def on_epoch_ended(self):
        self.increment_epoch()


class DecisionGD(DecisionBase):
    """Classification decision (error percentage per class)."""
    MAPPING = "decision_gd"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.epoch_n_err = [0.0, 0.0, 0.0]
        self.epoch_n_err_pt = [100.0, 100.0, 100.0]
        self.epoch_loss = [0.0, 0.0, 0.0]
        self.min_validation_n_err_pt = 1e30
        self.min_train_n_err_pt = 1e30
        self.best_epoch = -1
        self.history = []
        self.demand("evaluator")

    def on_last_minibatch(self, cls):
        m = self.evaluator.take_class_metrics(cls)
        m = self.dp_all_reduce(m).cpu().numpy().astype(numpy.float64)
        n = max(m[2], 1.0)
        self.epoch_n_err[cls] = m[0]
        self.epoch_n_err_pt[cls] = 100.0 * m[0] / n
        self.epoch_loss[cls] = m[1] / n
        if hasattr(self.evaluator, "take_confusion"):
            self.evaluator.take_confusion(
                cls, shown=cls == VALID or (cls == TRAIN and
                                            self.class_lengths[VALID] == 0))

    def on_epoch_ended(self):
        has_valid = self.class_lengths[VALID] > 0
        key = VALID if has_valid else TRAIN
        err = self.epoch_n_err_pt[key]
        self.improved <<= err < self.min_validation_n_err_pt
        if self.improved:
            self.min_validation_n_err_pt = err
            self.best_epoch = self.epoch_number
            self._fails = 0
        else:
            self._fails += 1
        tr = self.epoch_n_err_pt[TRAIN]
        self.train_improved <<= tr < self.min_train_n_err_pt
        if self.train_improved:
            self.min_train_n_err_pt = tr
        self.snapshot_suffix = "%s_%.2f_train_%.2f" % (
            CLASS_NAME[key], err, tr)
        self.history.append({
            "epoch": self.epoch_number,
            "validation_err_pt": self.epoch_n_err_pt[VALID],
            "train_err_pt": tr, "test_err_pt": self.epoch_n_err_pt[TEST],
            "validation_loss": self.epoch_loss[VALID],
            "train_loss": self.epoch_loss[TRAIN]})
        self.info("Epoch %d: validation %.2f%% train %.2f%% (loss %.4f / "
                  "%.4f)%s", self.epoch_number, self.epoch_n_err_pt[VALID],
                  tr, self.epoch_loss[VALID], self.epoch_loss[TRAIN],
                  " *" if self.improved else "")
        if self.fail_iterations is not None and \
                self._fails >= self.fail_iterations:
            self.complete <<= True
        self.increment_epoch()

    def get_metric_names(self):
        return {"Best validation error", "Best epoch", "EvaluationFitness",
                "Train error", "Epoch history"}

    def get_metric_values(self):
        best = self.min_validation_n_err_pt
        return {"Best validation error": best,
                "Best epoch": self.best_epoch,
                "Train error": self.epoch_n_err_pt[TRAIN],
                "EvaluationFitness": 1.0 - min(best, 100.0) / 100.0,
                "Epoch history": self.history}


class DecisionMSE(DecisionBase):
    MAPPING = "decision_mse"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.epoch_mse = [0.0, 0.0, 0.0]
        self.epoch_rmse = [0.0, 0.0, 0.0]
        self.min_validation_mse = 1e30
        self.best_epoch = -1
        self.history = []
        self.demand("evaluator")

    def on_last_minibatch(self, cls):
        m = self.evaluator.take_class_metrics(cls)
        m = self.dp_all_reduce(m).cpu().numpy().astype(numpy.float64)
        n = max(m[2], 1.0)
        self.epoch_mse[cls] = m[0] / n
        self.epoch_rmse[cls] = m[1] / n

    def on_epoch_ended(self):
        key = VALID if self.class_lengths[VALID] > 0 else TRAIN
        v = self.epoch_mse[key]
        self.improved <<= v < self.min_validation_mse
        if self.improved:
            self.min_validation_mse = v
            self.best_epoch = self.epoch_number
            self._fails = 0
        else:
            self._fails += 1
        self.snapshot_suffix = "%s_%.6f" % (CLASS_NAME[key], v)
        self.history.append({"epoch": self.epoch_number, "mse": v,
                             "train_mse": self.epoch_mse[TRAIN]})
        self.info("Epoch %d: validation mse %.6f rmse %.6f train mse %.6f",
                  self.epoch_number, v, self.epoch_rmse[key],
                  self.epoch_mse[TRAIN])
        if self._fails >= (self.fail_iterations or 1e30):
            self.complete <<= True
        self.increment_epoch()

    def get_metric_values(self):
        return {"Best validation MSE": self.min_validation_mse,
                "Best epoch": self.best_epoch,
                "EvaluationFitness": 1.0 / (1.0 + self.min_validation_mse),
                "Epoch history": self.history}
