"""Backward units of the fully connected layers (Znicz ``gd.py`` family).

grad_W[out][in] += err^T . x        (MFMA GEMM, TN layout, f32 accumulate)
grad_b[out]     += colsum(err)      (hvk_col_sum)
err_input       =  err . W  [* f'(below.output)]   (GEMM, NN layout, fused
                                                    derivative epilogue)
where err = err_output * f'(output) unless the unit above already fused it.
"""
from __future__ import annotations

from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops

__all__ = ["GradientDescent", "GDTanh", "GDRELU", "GDStrictRELU",
           "GDSigmoid", "GDSoftmax"]


def _bias_colsum():
    """FC bias gradient by ops.col_sum instead of the fused ones column
    (root.common.engine.fc_bias_colsum / VELES_AMD_FC_BIAS_COLSUM)."""
    import os
    from veles_amd.utils.config import root, get
    return os.environ.get("VELES_AMD_FC_BIAS_COLSUM", "1" if get(
        root.common.engine.fc_bias_colsum, False) else "0") != "0"


class GradientDescent(GradientDescentBase):
    MAPPING = "all2all"
    OVERWRITES_GRADS = True  # see ParameterStore.overwrite

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        fwd = self.forward
        if fwd is None:
            raise AttributeError("%s: forward_unit is not set" % self)
        self.attach_params(fwd)

    def run(self):
        fwd = self.forward
        fwd.ensure_params()
        err = self.err_output_effective()
        B = err.shape[0]
        e2 = err.reshape(B, -1)
        x = self.input.devmem.reshape(B, -1)
        if x.dtype != e2.dtype:
            x = x.to(e2.dtype)
        pw, pb = fwd._pw_, fwd._pb_
        bg = None if pb is None else pb.grad
        # the step's only contribution: write, not read-modify-write
        ow = self.store_.overwrite
        mode = "overwrite" if ow else True
        if not fwd.weights_transposed and bg is not None and \
                _bias_colsum() and e2.is_cuda:
            # grad_b by the column-sum kernel: the ones column costs the
            # weight-gradient GEMM one more column tile and its buffer-DMA
            # path (engine.fc_bias_colsum)
            ops.gemm(e2, x, trans_a=True, out=pw.grad, accumulate=mode)
            ops.col_sum(e2, out=bg, accumulate=not ow)
        elif not fwd.weights_transposed:
            # grad_W and grad_b (ones column) from one GEMM
            ops.gemm(e2, x, trans_a=True, out=pw.grad, accumulate=mode,
                     bias_grad=bg)
        else:
            ops.gemm(x, e2, trans_a=True, out=pw.grad, accumulate=mode)
            if bg is not None:
                ops.col_sum(e2, out=bg, accumulate=not ow)
        if self.need_err_input:
            ei = self.alloc_err_input(self.input.devmem.shape)
            aux, aux_act = self.aux_tensor()
            aux2 = None if aux is None else aux.reshape(B, -1)
            # stays bf16 under float8 as well: an fp8 dgrad would need W^T
            # materialised every step, which costs more than the GEMM
            ops.gemm(e2, fwd.weights_lp, trans_b=fwd.weights_transposed,
                     out=ei.view(B, -1), aux=aux2, aux_act=aux_act)
        self.report_gradients()


class GDTanh(GradientDescent):
    MAPPING = "all2all_tanh"


class GDRELU(GradientDescent):
    MAPPING = "all2all_relu"


class GDStrictRELU(GradientDescent):
    MAPPING = "all2all_str"


class GDSigmoid(GradientDescent):
    MAPPING = "all2all_sigmoid"


class GDSoftmax(GradientDescent):
    MAPPING = "softmax"
