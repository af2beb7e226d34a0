"""Backward units of the convolutional layers (Znicz ``gd_conv``).

grad_W += wgrad(x, err)   implicit-GEMM MFMA, split over pixels, f32 atomics
grad_b += colsum(err)
err_input = dgrad(err, W) [* f'(below.output)]  implicit transposed-conv GEMM
            (fp8: e5m2 err x e4m3 W on the fp8 MFMA kernel when the forward
            layer runs in fp8; the weight gradient stays bf16)
"""
from __future__ import annotations

from veles_amd.models.conv import input_tensor
from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops
from veles_amd.ops import fp8

__all__ = ["GradientDescentConv", "GDTanhConv", "GDRELUConv",
           "GDStrictRELUConv", "GDSigmoidConv"]


class GradientDescentConv(GradientDescentBase):
    MAPPING = "conv"
    OVERWRITES_GRADS = True  # starts from a zeroed span, then accumulates
    ZEROED_BY_UPDATE = True  # the fused update clears the span for it

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        if self.forward is None:
            raise AttributeError("%s: forward_unit is not set" % self)
        self.attach_params(self.forward)

    def init_unpickled(self):
        super().init_unpickled()
        self.fp8_sdy_ = None
        self.dy8_ = None

    def run(self):
        fwd = self.forward
        fwd.ensure_params()
        err = self.err_output_effective()
        x = input_tensor(self.input)
        s2d = isinstance(x, ops.S2DImage)   # loader-made s2d input
        squeeze = not s2d and x.dim() == 3
        if squeeze:
            x = x.unsqueeze(-1)
        if not s2d and x.dtype != err.dtype:
            x = x.to(err.dtype)
        pw, pb = fwd._pw_, fwd._pb_
        if self.store_.overwrite and not all(
                self.store_.cleared_by_update(p) for p in (pw, pb)
                if p is not None):
            # the split-K atomics of this layer start from its own zeroed
            # span (normally the update already cleared it: zero_tail)
            self.store_.zero_grads((pw, pb))
        # weight AND bias gradients from one implicit-GEMM launch
        ops.conv_wgrad(x, err, pw.grad, fwd.sliding, fwd.padding,
                       fwd.grouping, col=getattr(fwd, "col_", None),
                       dbias=None if pb is None else pb.grad)
        if self.need_err_input:
            ei = self.alloc_err_input(tuple(x.shape))
            aux, aux_act = self.aux_tensor()
            if aux is not None and aux.dim() == 3:
                aux = aux.unsqueeze(-1)
            if getattr(fwd, "fp8_", False):
                # e5m2 gradient x e4m3 weights on the fp8 MFMA kernel
                if self.fp8_sdy_ is None:
                    self.fp8_sdy_ = fp8.Scaler(self.torch_device, fp8.E5M2)
                self.dy8_ = fp8.quantize(err, self.fp8_sdy_, out=self.dy8_)
                wt8 = fp8.permute_for_dgrad(fwd.w8_, fwd.grouping) \
                    if err.is_cuda else None
                fp8.conv_dgrad(self.dy8_, self.fp8_sdy_, fwd.w8_,
                               fwd.fp8_sw_, tuple(x.shape), fwd.sliding,
                               fwd.padding, fwd.grouping, aux=aux,
                               aux_act=aux_act, out=ei, wt8=wt8)
            else:
                ops.conv_dgrad(err, fwd.weights_lp, tuple(x.shape),
                               fwd.sliding, fwd.padding, fwd.grouping,
                               aux=aux, aux_act=aux_act, out=ei)
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
