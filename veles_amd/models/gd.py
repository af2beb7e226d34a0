"""Backward units of the fully connected layers (Znicz ``gd.py`` family).

grad_W[out][in] += err^T . x        (MFMA GEMM, TN layout, f32 accumulate)
grad_b[out]     += colsum(err)      (hvk_col_sum)
err_input       =  err . W  [* f'(below.output)]   (GEMM, NN layout, fused
                                                    derivative epilogue)
where err = err_output * f'(output) unless the unit above already fused it.

Under precision_type "float8" the backward-data of an fp8 layer runs on the
fp8 MFMA too (round 4): err quantised to e5m2, against an e4m3 W^T made by
transposing the forward's weight copy (same scaler) - the fp8 GEMM takes
K-major operands only.  ``root.common.engine.fp8_fc_dgrad = False`` keeps
the bf16 GEMM.
"""
from __future__ import annotations

import torch

from veles_amd.models.nn_units import GradientDescentBase
from veles_amd import ops
from veles_amd.ops import fp8
from veles_amd.models.gd_conv import _side_stream_run, _wgrad_on_side

__all__ = ["GradientDescent", "GDTanh", "GDRELU", "GDStrictRELU",
           "GDSigmoid", "GDSoftmax"]


def _bias_colsum():
    """FC bias gradient by ops.col_sum instead of the fused ones column
    (root.common.engine.fc_bias_colsum / VELES_AMD_FC_BIAS_COLSUM)."""
    import os
    from veles_amd.utils.config import root, get
    return os.environ.get("VELES_AMD_FC_BIAS_COLSUM", "1" if get(
        root.common.engine.fc_bias_colsum, False) else "0") != "0"


def _wgrad_nn(e2, x):
    """FC weight gradient as transpose + NN GEMM (GPU bf16, batch and
    outputs multiples of 64; root.common.engine.fc_wgrad_nn /
    VELES_AMD_FC_WGRAD_NN, on by default: AlexNet b3072 fc6 / fc7,
    profiles/r6/fc_wgrad_nn_r6kk.log)."""
    if not e2.is_cuda or e2.dtype != torch.bfloat16 or \
            x.dtype != torch.bfloat16 or e2.shape[0] % 64 or \
            e2.shape[1] % 64 or not e2.is_contiguous() or \
            not x.is_contiguous():
        return False
    import os
    from veles_amd.utils.config import root, get
    return os.environ.get("VELES_AMD_FC_WGRAD_NN", "1" if get(
        root.common.engine.fc_wgrad_nn, True) else "0") != "0"


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
        tmp = ()
        if x.dtype != e2.dtype:
            x = x.to(e2.dtype)
            tmp = (x,)
        pw, pb = fwd._pw_, fwd._pb_
        bg = None if pb is None else pb.grad
        # the step's only contribution: write, not read-modify-write
        ow = self.store_.overwrite
        mode = "overwrite" if ow else True

        def wgrad():
            if not fwd.weights_transposed and _wgrad_nn(e2, x):
                # dY^T (and the bias gradient) in one pass, then the NN
                # GEMM: K-major A takes the 256 x 128 ping-pong loop, which
                # the MN-major dY of the TN form (and its ones column) miss
                R, C = e2.shape
                if self.e2t_ is None or self.e2t_.shape != (C, R):
                    self.e2t_ = torch.empty(C, R, dtype=e2.dtype,
                                            device=e2.device)
                    self.e2t_ws_ = torch.empty(R // 64 * C,
                                               dtype=torch.float32,
                                               device=e2.device)
                ops.transpose_colsum(e2, out=self.e2t_, colsum=bg,
                                     accumulate=not ow, ws=self.e2t_ws_)
                ops.gemm(self.e2t_, x, out=pw.grad, accumulate=mode)
            elif not fwd.weights_transposed and bg is not None and \
                    _bias_colsum() and e2.is_cuda:
                # grad_b by the column-sum kernel: the ones column costs the
                # weight-gradient GEMM one more column tile and its
                # buffer-DMA path (engine.fc_bias_colsum)
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

        if _wgrad_on_side(self, e2):
            # off the compute stream, under the backward-data chain below
            # (gd_conv.py)
            _side_stream_run(self, wgrad, keep=tmp)
        else:
            wgrad()
        if self.need_err_input:
            ei = self.alloc_err_input(self.input.devmem.shape)
            aux, aux_act = self.aux_tensor()
            aux2 = None if aux is None else aux.reshape(B, -1)
            if self._fp8_dgrad_ok(fwd):
                self._fp8_dgrad(fwd, e2, ei.view(B, -1), aux2, aux_act)
            else:
                ops.gemm(e2, fwd.weights_lp, trans_b=fwd.weights_transposed,
                         out=ei.view(B, -1), aux=aux2, aux_act=aux_act)
        self.report_gradients()

    def init_unpickled(self):
        super().init_unpickled()
        self.e8_ = self.wt8_ = self.fp8_se_ = None
        self.e2t_ = self.e2t_ws_ = None

    def __getstate__(self):
        fp8.save_scalers(self, ("fp8_se_",))
        return super().__getstate__()

    def _fp8_dgrad_ok(self, fwd):
        from veles_amd.utils.config import root, get
        return getattr(fwd, "fp8_", False) and \
            getattr(fwd, "w8_", None) is not None and \
            get(root.common.engine.fp8_fc_dgrad, True)

    def _fp8_dgrad(self, fwd, e2, out, aux, aux_act):
        """err_input = deq(e5m2(err)) . deq(e4m3(W)) on the fp8 MFMA: the
        forward's e4m3 weight copy transposed once per step into a K-major
        [in][out] image (the scale is the copy's)"""
        if self.fp8_se_ is None:
            self.fp8_se_ = fp8.Scaler(e2.device, fp8.E5M2)
            fp8.restore_scaler(self, "fp8_se_")
        self.e8_ = fp8.quantize(e2, self.fp8_se_, out=self.e8_)
        w8 = fwd.w8_
        if self.wt8_ is None or self.wt8_.shape != (w8.shape[1], w8.shape[0]):
            self.wt8_ = torch.empty(w8.shape[1], w8.shape[0], dtype=w8.dtype,
                                    device=w8.device)
        self.wt8_.view(torch.uint8).copy_(w8.view(torch.uint8).t())
        fp8.gemm(self.e8_, self.fp8_se_, self.wt8_, fwd.fp8_sw_, aux=aux,
                 aux_act=aux_act, out=out)


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
