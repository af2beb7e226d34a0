"""Standalone activation units (Znicz ``activation_*`` types).

tanh / relu (softplus) / strict relu / sigmoid run as ``hvk_act_fwd`` /
``hvk_act_bwd``.  log (y = log(x + sqrt(x^2 + 1)), i.e. asinh), tanhlog
(tanh for |x| <= 1 region, log growth beyond - docs/OPS.md), sincos (even
outputs sin, odd cos) and mul (y = k x) are composed from device tensor ops.
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

    def compute(self, x):
        raise NotImplementedError

    def run(self):
        x = self.input.devmem
        if self.ACT:
            ops.act_fwd(x, self.ACT, out=self._alloc(x))
        else:
            self._alloc(x).copy_(self.compute(x.float()).to(x.dtype))


class ActivationBackward(GradientDescentBase):
    hide_from_registry = True
    ACT = 0

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("output")

    def derivative(self, x, y):
        raise NotImplementedError

    def run(self):
        err = self.err_output.devmem
        ei = self.alloc_err_input(tuple(err.shape), err.dtype)
        if self.ACT:
            ops.act_bwd(err, self.output.devmem, self.ACT, out=ei)
        else:
            d = self.derivative(self.input.devmem.float(),
                                self.output.devmem.float())
            ei.copy_((err.float() * d).to(ei.dtype))
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

    def compute(self, x):
        return torch.log(x + torch.sqrt(x * x + 1))


class BackwardLog(ActivationBackward):
    MAPPING = "activation_log"

    def derivative(self, x, y):
        return 1.0 / torch.sqrt(x * x + 1)


class ForwardTanhLog(ActivationForward):
    MAPPING = "activation_tanhlog"
    D = 0.9

    def compute(self, x):
        a = x.abs()
        lin = 1.7159 * torch.tanh(0.6666 * x)
        edge = 1.7159 * torch.tanh(torch.tensor(0.6666 * self.D))
        slope = 1.7159 * 0.6666 * (1 - torch.tanh(
            torch.tensor(0.6666 * self.D)) ** 2)
        logp = torch.sign(x) * (edge + slope * self.D * torch.log(
            a.clamp(min=self.D) / self.D))
        return torch.where(a <= self.D, lin, logp)


class BackwardTanhLog(ActivationBackward):
    MAPPING = "activation_tanhlog"
    D = 0.9

    def derivative(self, x, y):
        a = x.abs()
        t = torch.tanh(0.6666 * x)
        dlin = 1.7159 * 0.6666 * (1 - t * t)
        slope = 1.7159 * 0.6666 * (1 - torch.tanh(
            torch.tensor(0.6666 * self.D)) ** 2)
        dlog = slope * self.D / a.clamp(min=self.D)
        return torch.where(a <= self.D, dlin, dlog)


class ForwardSinCos(ActivationForward):
    MAPPING = "activation_sincos"

    def compute(self, x):
        flat = x.reshape(x.shape[0], -1)
        out = torch.empty_like(flat)
        out[:, 0::2] = torch.sin(flat[:, 0::2])
        out[:, 1::2] = torch.cos(flat[:, 1::2])
        return out.view(x.shape)


class BackwardSinCos(ActivationBackward):
    MAPPING = "activation_sincos"

    def derivative(self, x, y):
        flat = x.reshape(x.shape[0], -1)
        d = torch.empty_like(flat)
        d[:, 0::2] = torch.cos(flat[:, 0::2])
        d[:, 1::2] = -torch.sin(flat[:, 1::2])
        return d.view(x.shape)


class ForwardMul(ActivationForward):
    MAPPING = "activation_mul"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.factor = kwargs.get("factor", 1.0)

    def compute(self, x):
        return x * self.factor


class BackwardMul(ActivationBackward):
    MAPPING = "activation_mul"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.factor = kwargs.get("factor", 1.0)

    def derivative(self, x, y):
        return torch.full_like(x, self.factor)
