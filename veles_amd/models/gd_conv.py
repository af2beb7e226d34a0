"""Backward units of the convolutional layers (Znicz ``gd_conv``).

grad_W += wgrad(x, err)   implicit-GEMM MFMA, split over pixels, f32 atomics
grad_b += colsum(err)
err_input = dgrad(err, W) [* f'(below.output)]  implicit transposed-conv GEMM
"""
from __future__ import annotations

from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops

__all__ = ["GradientDescentConv", "GDTanhConv", "GDRELUConv",
           "GDStrictRELUConv", "GDSigmoidConv"]


class GradientDescentConv(GradientDescentBase):
    MAPPING = "conv"

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        if self.forward is None:
            raise AttributeError("%s: forward_unit is not set" % self)
        self.attach_params(self.forward)

    def run(self):
        fwd = self.forward
        fwd.ensure_params()
        err = self.err_output_effective()
        x = self.input.devmem
        squeeze = x.dim() == 3
        if squeeze:
            x = x.unsqueeze(-1)
        if x.dtype != err.dtype:
            x = x.to(err.dtype)
        pw, pb = fwd._pw_, fwd._pb_
        # weight AND bias gradients from one implicit-GEMM launch
        ops.conv_wgrad(x, err, pw.grad, fwd.sliding, fwd.padding,
                       fwd.grouping, col=getattr(fwd, "col_", None),
                       dbias=None if pb is None else pb.grad)
        if self.need_err_input:
            ei = self.alloc_err_input(tuple(x.shape))
            aux, aux_act = self.aux_tensor()
            if aux is not None and aux.dim() == 3:
                aux = aux.unsqueeze(-1)
            ops.conv_dgrad(err, fwd.weights_lp, tuple(x.shape), fwd.sliding,
                           fwd.padding, fwd.grouping, aux=aux,
                           aux_act=aux_act, out=ei)
            if squeeze:
                self.err_input.devmem = ei.squeeze(-1)
        self.report_gradients()


class GDTanhConv(GradientDescentConv):
    MAPPING = "conv_tanh"


class GDRELUConv(GradientDescentConv):
    MAPPING = "conv_relu"


class GDStrictRELUConv(GradientDescentConv):
    MAPPING = "conv_str"


class GDSigmoidConv(GradientDescentConv):
    MAPPING = "conv_sigmoid"
