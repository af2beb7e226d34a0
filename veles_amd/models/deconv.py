"""Deconvolution (transposed convolution) and its backward unit (Znicz
``deconv.Deconv`` / ``gd_deconv.GDDeconv``, listed in
docs/source/manualrst_veles_workflow_parameters.rst:477).

Weights are laid out like the Conv that this layer inverts:
[n_kernels][ky][kx][n_channels] where ``n_kernels`` is the channel count of
the deconv INPUT and ``n_channels`` of its output.  On the MI355X:

* forward  y  = conv^T(x, W)           -> ``hvk_conv_dgrad`` (implicit GEMM)
* err_input   = conv(err_output, W)    -> ``hvk_conv_fwd``
* grad_W     += wgrad(err_output, x)   -> ``hvk_conv_wgrad`` (split-K, f32)

so the three directions of a deconv reuse the three MFMA conv kernels with
the roles of input and output exchanged.
"""
from __future__ import annotations

import torch

from veles_amd.models.conv import norm_padding, norm_sliding
from veles_amd.models.nn_units import Forward, GradientDescentBase
from veles_amd import ops

__all__ = ["Deconv", "GDDeconv"]


class Deconv(Forward):
    __id__ = "6a8c1c9e-5d0e-4d5c-9a43-3b1f0f6a2d11"
    MAPPING = "deconv"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("include_bias", False)
        super().__init__(workflow, **kwargs)
        self.n_kernels = int(kwargs["n_kernels"])
        self.kx = int(kwargs["kx"])
        self.ky = int(kwargs["ky"])
        self.padding = norm_padding(kwargs.get("padding"))
        self.sliding = norm_sliding(kwargs.get("sliding"))
        self.n_channels = kwargs.get("n_channels")
        self.unsafe_padding = kwargs.get("unsafe_padding", False)
        # optional: a unit whose ``input`` shape the output must match
        # (the Conv being inverted in an auto-encoder)
        self.output_shape_source = kwargs.get("output_shape_source")

    def out_shape(self, in_shape):
        N, H, W, K = in_shape
        src = self.output_shape_source
        if src is not None:
            shp = tuple(getattr(src, "input", src).shape)
            if len(shp) == 3:
                shp = shp + (1,)
            return (N,) + tuple(shp[1:])
        if self.n_channels is None:
            raise ValueError("%s: set n_channels or output_shape_source" %
                             self)
        pl, pt, pr, pb = self.padding
        sx, sy = self.sliding
        return (N, (H - 1) * sy + self.ky - pt - pb,
                (W - 1) * sx + self.kx - pl - pr, int(self.n_channels))

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        shape = tuple(self.input.shape)
        if len(shape) == 3:
            shape = shape + (1,)
        if shape[3] != self.n_kernels:
            raise ValueError("%s: input has %d channels, n_kernels is %d" %
                             (self, shape[3], self.n_kernels))
        oshape = self.out_shape(shape)
        OH, OW = ops.conv_out_size(oshape[1], oshape[2], self.ky, self.kx,
                                   self.sliding, self.padding)
        if (OH, OW) != shape[1:3]:
            raise ValueError("%s: output %s does not convolve back to %s" %
                             (self, oshape, shape))
        C = oshape[3]
        self.register_params((self.n_kernels, self.ky, self.kx, C),
                             self.ky * self.kx * self.n_kernels)
        self.out_shape_ = oshape
        self.alloc_output(oshape)

    def run(self):
        x = self.input.devmem
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        y = self.alloc_output(self.out_shape_)
        if x.dtype != self.weights_lp.dtype:
            x = x.to(self.weights_lp.dtype)
        ops.conv_dgrad(x, self.weights_lp, self.out_shape_, self.sliding,
                       self.padding, 1, out=y)
        if self.include_bias:
            y += self.bias_master.to(y.dtype)

    def package_export(self):
        d = super().package_export()
        d.update({"kx": self.kx, "ky": self.ky, "n_kernels": self.n_kernels,
                  "padding": list(self.padding),
                  "sliding": list(self.sliding)})
        return d


class GDDeconv(GradientDescentBase):
    MAPPING = "deconv"

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
        ops.conv_wgrad(err, x, pw.grad, fwd.sliding, fwd.padding, 1)
        if pb is not None:
            ops.col_sum(err.reshape(-1, err.shape[-1]), out=pb.grad,
                        accumulate=True)
        if self.need_err_input:
            ei = self.alloc_err_input(tuple(x.shape))
            ops.conv_fwd(err, fwd.weights_lp, None, fwd.sliding, fwd.padding,
                         1, 0, out=ei)
            aux, aux_act = self.aux_tensor()
            if aux is not None:
                ops.act_bwd(ei, aux.reshape(ei.shape), aux_act, out=ei)
            if squeeze:
                self.err_input.devmem = ei.squeeze(-1)
        self.report_gradients()


_ = torch  # imported for type use in subclasses
