"""Convolutional layers (Znicz ``conv*`` types; docs/OPS.md §Conv).

NHWC input [B, H, W, C]; weights [n_kernels][ky][kx][C/grouping];
``padding`` = (left, top, right, bottom), ``sliding`` = (x, y).  Forward is
one implicit-GEMM MFMA kernel (``hvk_conv_fwd``: im2col gathered on the fly
from NHWC, bias + activation in the epilogue, groups on grid z).  With
``precision_type = "float8"`` and 16-aligned channel counts the input and
weights are quantized to e4m3 and the conv runs on the fp8 MFMA kernel
(``hvk_conv_fwd_fp8``, veles_amd/ops/fp8.py).
"""
from __future__ import annotations

from veles_amd.models.nn_units import Forward
from veles_amd import ops
from veles_amd.ops import fp8

__all__ = ["Conv", "input_shape", "input_tensor", "ConvTanh", "ConvRELU", "ConvStrictRELU", "ConvSigmoid",
           "norm_padding", "norm_sliding"]


def norm_padding(p):
    if p is None:
        return (0, 0, 0, 0)
    if isinstance(p, int):
        return (p, p, p, p)
    p = tuple(p)
    if len(p) == 2:
        return (p[0], p[1], p[0], p[1])
    return p


def norm_sliding(s):
    if s is None:
        return (1, 1)
    if isinstance(s, int):
        return (s, s)
    return tuple(s)


def input_shape(arr):
    """Logical NHWC shape of a conv input Array (the loader may serve it in
    space-to-depth layout: ``Array.s2d_``)."""
    spec = getattr(arr, "s2d_", None)
    return tuple(spec[1]) if spec is not None else tuple(arr.shape)


def input_tensor(arr):
    """The device tensor of a conv input Array, wrapped as ops.S2DImage when
    the loader serves it in space-to-depth layout."""
    spec = getattr(arr, "s2d_", None)
    if spec is not None:
        return ops.S2DImage(arr.devmem, spec[0], spec[1])
    return arr.devmem


class Conv(Forward):
    __id__ = "bd4f8f3d-0a43-4a8e-b4d5-5b1b9d3a1c10"
    MAPPING = "conv"
    ACTIVATION = 0

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.n_kernels = int(kwargs["n_kernels"])
        self.kx = int(kwargs["kx"])
        self.ky = int(kwargs["ky"])
        self.padding = norm_padding(kwargs.get("padding"))
        self.sliding = norm_sliding(kwargs.get("sliding"))
        self.grouping = int(kwargs.get("grouping", 1))
        self.unsafe_padding = kwargs.get("unsafe_padding", False)

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        self._request_s2d_input()
        shape = input_shape(self.input)
        if len(shape) == 3:
            shape = tuple(shape) + (1,)
        self.in_shape_ = shape
        C = shape[3]
        if C % self.grouping or self.n_kernels % self.grouping:
            raise ValueError("%s: channels %d / kernels %d not divisible by "
                             "grouping %d" % (self, C, self.n_kernels,
                                              self.grouping))
        cg = C // self.grouping
        self.register_params((self.n_kernels, self.ky, self.kx, cg),
                             self.ky * self.kx * cg)
        OH, OW = self.output_hw(shape[1], shape[2])
        self.alloc_output((shape[0], OH, OW, self.n_kernels))
        self.fp8_ = bool(getattr(self.device, "fp8", False)) and \
            fp8.fp8_conv_ok(C, self.n_kernels, self.grouping, self.ky,
                             self.kx) and fp8.fp8_conv_pays(C, OH, OW)
        if self.fp8_ and self.fp8_sx_ is None:
            self.fp8_sx_ = fp8.Scaler(self.torch_device, fp8.E4M3)
            self.fp8_sw_ = fp8.Scaler(self.torch_device, fp8.E4M3)
            fp8.restore_scaler(self, "fp8_sx_")
            fp8.restore_scaler(self, "fp8_sw_")

    def __getstate__(self):
        fp8.save_scalers(self, ("fp8_sx_", "fp8_sw_"))
        return super().__getstate__()

    def init_unpickled(self):
        super().init_unpickled()
        self.col_ = None
        self.fp8_ = False
        self.fp8_sx_ = self.fp8_sw_ = None
        self.x8_ = self.w8_ = None
        # fused input quantisation: the producing conv wrote x8_ this pass
        self.x8_fresh_ = False
        self.q8_consumer_ = None

    def fp8_input_consumer(self):
        return fp8_input_consumer(self)

    def _q8_target(self, y):
        return fp8_input_target(self, y)

    def output_hw(self, H, W):
        return ops.conv_out_size(H, W, self.ky, self.kx, self.sliding,
                                 self.padding)

    # units besides the forwards that read the loader's minibatch_data as
    # an NHWC image: with any of them the s2d input layout stays off
    _IMAGE_READERS = ("avatar", "data_saver", "image_saver",
                      "immediate_plotter", "meandispnorm")

    def _request_s2d_input(self):
        """First layer, strided RGB conv (AlexNet conv1): ask the loader to
        gather straight into this conv's space-to-depth layout, saving the
        bf16 image's write + read and the separate s2d pass
        (``root.common.engine.fuse_input_layout``, default on)."""
        from veles_amd.utils.config import root, get
        wf = self.workflow
        ld = getattr(wf, "loader", None)
        if getattr(self.input, "s2d_", None) is not None:
            return
        if ld is None or self.input is not ld.minibatch_data or \
                not hasattr(ld, "request_s2d_input") or \
                not get(root.common.engine.fuse_input_layout, True) or \
                not getattr(self.device, "is_gpu", False) or \
                getattr(self.device, "fp8", False) or \
                any(getattr(wf, a, None) is not None
                    for a in self._IMAGE_READERS):
            return
        shape = tuple(self.input.shape)
        if len(shape) != 4:
            return
        s = ops.s2d_factor(shape[3], self.grouping, self.sliding, self.ky,
                           self.kx)
        if s and ld.request_s2d_input(s, self.ky, self.kx, self.padding):
            self.info("input served in space-to-depth layout (s = %d) by "
                      "the loader's fused gather", s)

    def run(self):
        x = input_tensor(self.input)
        if isinstance(x, ops.S2DImage):
            B, H, W, C = x.shape
            OH, OW = self.output_hw(H, W)
            y = self.alloc_output((B, OH, OW, self.n_kernels))
            ws = {}
            ops.conv_fwd(x, self.weights_lp, self.bias_master, self.sliding,
                         self.padding, self.grouping, self.activation, out=y,
                         col_out=ws)
            self.col_ = ws.get("col")
            return
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        B, H, W, C = x.shape
        OH, OW = self.output_hw(H, W)
        y = self.alloc_output((B, OH, OW, self.n_kernels))
        if self.fp8_:
            # e4m3 input and weights, delayed per-tensor scaling (ops/fp8.py);
            # the input copy comes from the producing conv's epilogue when
            # that conv wrote it this pass (x8_fresh_)
            if not self.x8_fresh_ or self.x8_ is None or \
                    tuple(self.x8_.shape) != tuple(x.shape):
                self.x8_ = fp8.quantize(x, self.fp8_sx_, out=self.x8_)
            self.x8_fresh_ = False
            self.w8_ = fp8.quantize(self.weights_lp, self.fp8_sw_,
                                    out=self.w8_)
            q8, qs = self._q8_target(y)
            fp8.conv_fwd(self.x8_, self.fp8_sx_, self.w8_, self.fp8_sw_,
                         self.bias_master, self.sliding, self.padding,
                         self.grouping, self.activation, out=y, q8=q8,
                         q8_scaler=qs)
            if q8 is not None:
                self.fp8_input_consumer().x8_fresh_ = True
            return
        if x.dtype != self.weights_lp.dtype:
            x = x.to(self.weights_lp.dtype)
        ws = {}
        # a bf16 conv feeding an fp8 conv (VGG conv1_1, C = 3) writes that
        # conv's e4m3 input copy from its epilogue too
        q8, qs = self._q8_target(y)
        ops.conv_fwd(x, self.weights_lp, self.bias_master, self.sliding,
                     self.padding, self.grouping, self.activation, out=y,
                     col_out=ws, q8=q8, q8_scaler=qs)
        if q8 is not None:
            self.fp8_input_consumer().x8_fresh_ = True
        self.col_ = ws.get("col")

    def package_export(self):
        d = super().package_export()
        d.update({"kx": self.kx, "ky": self.ky, "n_kernels": self.n_kernels,
                  "padding": list(self.padding),
                  "sliding": list(self.sliding), "grouping": self.grouping})
        return d


class ConvTanh(Conv):
    MAPPING = "conv_tanh"
    ACTIVATION = 1


class ConvRELU(Conv):
    MAPPING = "conv_relu"
    ACTIVATION = 2


class ConvStrictRELU(Conv):
    MAPPING = "conv_str"
    ACTIVATION = 3


class ConvSigmoid(Conv):
    MAPPING = "conv_sigmoid"
    ACTIVATION = 4


def fp8_input_consumer(unit):
    """The fp8 conv that reads ``unit``'s output as its input (direct link,
    no unit in between), or None: ``unit`` then also writes that conv's e4m3
    input copy from the kernel producing its output (fused quantisation:
    ``fp8.conv_fwd(q8=...)``, ``ops.pool2_fwd(q8=...)``)."""
    c = getattr(unit, "q8_consumer_", None)
    if c is None:
        c = False
        for u in getattr(unit, "links_to", ()):
            if isinstance(u, Conv) and u.fp8_ and \
                    getattr(u, "input", None) is unit.output:
                c = u
                break
        unit.q8_consumer_ = c
    return c or None


def fp8_input_target(unit, y):
    """(x8 buffer, scaler) for ``unit``'s fused output quantisation when the
    consumer's scaler is primed (its first pass quantized and primed it) and
    its buffer matches ``y``; (None, None) otherwise or with
    ``root.common.engine.fp8_fuse_quant = False``.  The caller sets the
    consumer's ``x8_fresh_`` once the producing kernel is enqueued."""
    from veles_amd.utils.config import root, get
    if not get(root.common.engine.fp8_fuse_quant, True):
        return None, None
    c = fp8_input_consumer(unit)
    if c is None or not c.fp8_sx_.primed or c.x8_ is None or \
            tuple(c.x8_.shape) != tuple(y.shape) or c.x8_.device != y.device:
        return None, None
    return c.x8_, c.fp8_sx_
