"""Learning-rate schedules (Znicz ``lr_adjust``; policies exp / fixed /
step_exp / inv / arbitrary_step, docs/source/manualrst_veles_workflow_
parameters.rst:669-680).  Runs once per TRAIN minibatch and rewrites the
``learning_rate`` / ``learning_rate_bias`` of its GD units; the fused SGD
kernel reads them through the segment table on the next update."""
from __future__ import annotations

from veles_amd.units import Unit

__all__ = ["LearningRateAdjust", "lr_policy"]


def lr_policy(name, base, **p):
    if name in (None, "fixed"):
        return lambda it: base
    if name == "exp":
        g = p.get("gamma", 0.9999)
        return lambda it: base * g ** it
    if name == "step_exp":
        g, step = p.get("gamma", 0.1), p.get("step", 10000)
        return lambda it: base * g ** (it // step)
    if name == "inv":
        g, pw = p.get("gamma", 1e-4), p.get("pow", 0.75)
        return lambda it: base * (1.0 + g * it) ** -pw
    if name == "arbitrary_step":
        steps = p.get("lrs_with_lengths", [(base, 1 << 62)])

        def f(it):
            acc = 0
            for lr, n in steps:
                acc += n
                if it < acc:
                    return lr
            return steps[-1][0]
        return f
    raise ValueError("Unknown lr policy %r" % name)


class LearningRateAdjust(Unit):
    MAPPING = "lr_adjust"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.lr_policy_name = kwargs.get("lr_policy_name", "fixed")
        self.bias_lr_policy_name = kwargs.get("bias_lr_policy_name",
                                              self.lr_policy_name)
        self.lr_parameters = kwargs.get("lr_parameters", {})
        self.bias_lr_parameters = kwargs.get("bias_lr_parameters",
                                             self.lr_parameters)
        self.gd_units = list(kwargs.get("gd_units", []))
        self.iteration = 0
        self.minibatch_class = 2

    def add_gd_unit(self, gd):
        self.gd_units.append(gd)

    def initialize(self, **kwargs):
        self._base = [(g.learning_rate, g.learning_rate_bias)
                      for g in self.gd_units]

    def run(self):
        if self.minibatch_class != 2:
            return
        self.iteration += 1
        for g, (lr, lrb) in zip(self.gd_units, self._base):
            g.learning_rate = lr_policy(self.lr_policy_name, lr,
                                        **self.lr_parameters)(self.iteration)
            g.learning_rate_bias = lr_policy(
                self.bias_lr_policy_name, lrb,
                **self.bias_lr_parameters)(self.iteration)
