"""Standalone activation units (Znicz ``activation_*`` types).

tanh / relu (softplus) / strict relu / sigmoid run as ``hvk_act_fwd`` /
``hvk_act_bwd`` (derivative through the output).  log (y = log(x +
sqrt(x^2 + 1)), i.e. asinh), tanhlog (scaled tanh up to |x| = D, log growth
beyond - docs/OPS.md), sincos (even feature columns sin, odd cos) and mul
(y = k x) differentiate through the INPUT: ``hvk_xact`` forward and
backward (ops.xact; float32 reference ops.xact_ref on the CPU).
"""
from __future__ import annotations

import torch

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops

__all__ = ["ActivationForward", "ActivationBackward", "ForwardTanh",
           "BackwardTanh", "ForwardRELU", "BackwardRELU", "ForwardStrictRELU",
           "BackwardStrictRELU", "ForwardSigmoid", "BackwardSigmoid",
           "ForwardLog", "BackwardLog", "ForwardTanhLog", "BackwardTanhLog",
           "ForwardSinCos", "BackwardSinCos", "ForwardMul", "BackwardMul"]


class ActivationForward(AcceleratedUnit):
    hide_from_registry = True
    ACT = 0

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.output = Array(shallow_pickle=True)
        self.demand("input")

    @property
    def activation(self):
        return 0  # derivative handled by the paired backward unit

    def package_export(self):
        return {"act": self.ACT}

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        import torch
        x = self.input.devmem
        self.output.devmem = torch.zeros(
            tuple(self.input.shape), dtype=x.dtype if x is not None else
            self.compute_dtype, device=self.torch_device)

    def _alloc(self, x):
        y = self.output.devmem
        if y is None or y.shape != x.shape or y.dtype != x.dtype or \
                y.device != x.device:
            self.output.devmem = y = torch.empty_like(x)
        return y

    XACT = None  # input-derivative kind (ops.XACT)

    def xact_param(self):
        return 0.0

    def compute(self, x):
        return ops.xact_ref(x, self.XACT, self.xact_param())

    def run(self):
        x = self.input.devmem
        if self.ACT:
            ops.act_fwd(x, self.ACT, out=self._alloc(x))
        else:
            ops.xact(x, self.XACT, self.xact_param(), out=self._alloc(x))


class ActivationBackward(GradientDescentBase):
    hide_from_registry = True
    ACT = 0

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("output")

    XACT = None

    def xact_param(self):
        return 0.0

    def derivative(self, x, y):
        return ops.xact_ref(x, self.XACT, self.xact_param(), bwd=True,
                            err=torch.ones_like(x))

    def run(self):
        err = self.err_output.devmem
        ei = self.alloc_err_input(tuple(err.shape), err.dtype)
        if self.ACT:
            ops.act_bwd(err, self.output.devmem, self.ACT, out=ei)
        else:
            ops.xact(self.input.devmem, self.XACT, self.xact_param(), out=ei,
                     err=err)
        aux, aux_act = self.aux_tensor()
        if aux is not None:
            ops.act_bwd(ei, aux, aux_act, out=ei)


def _pair(name, act, mapping):
    f = type("Forward" + name, (ActivationForward,),
             {"ACT": act, "MAPPING": "activation_" + mapping})
    b = type("Backward" + name, (ActivationBackward,),
             {"ACT": act, "MAPPING": "activation_" + mapping})
    return f, b


ForwardTanh, BackwardTanh = _pair("Tanh", 1, "tanh")
ForwardRELU, BackwardRELU = _pair("RELU", 2, "relu")
ForwardStrictRELU, BackwardStrictRELU = _pair("StrictRELU", 3, "str")
ForwardSigmoid, BackwardSigmoid = _pair("Sigmoid", 4, "sigmoid")


class ForwardLog(ActivationForward):
    MAPPING = "activation_log"
    XACT = "log"


class BackwardLog(ActivationBackward):
    MAPPING = "activation_log"
    XACT = "log"


class ForwardTanhLog(ActivationForward):
    MAPPING = "activation_tanhlog"
    XACT = "tanhlog"
    D = 0.9

    def xact_param(self):
        return self.D


class BackwardTanhLog(ActivationBackward):
    MAPPING = "activation_tanhlog"
    XACT = "tanhlog"
    D = 0.9

    def xact_param(self):
        return self.D


class ForwardSinCos(ActivationForward):
    MAPPING = "activation_sincos"
    XACT = "sincos"


class BackwardSinCos(ActivationBackward):
    MAPPING = "activation_sincos"
    XACT = "sincos"


class ForwardMul(ActivationForward):
    MAPPING = "activation_mul"
    XACT = "mul"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.factor = kwargs.get("factor", 1.0)

    def xact_param(self):
        return float(self.factor)


class BackwardMul(ActivationBackward):
    MAPPING = "activation_mul"
    XACT = "mul"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.factor = kwargs.get("factor", 1.0)

    def xact_param(self):
        return float(self.factor)
