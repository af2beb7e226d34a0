"""Backward units of the convolutional layers (Znicz ``gd_conv``).

grad_W (+)= wgrad(x, err)  stride 1: the halo kernel (wgrad_halo.hip), split
                         over pixels into workspace slices summed in split
                         order (deterministic); else the implicit-GEMM loop,
                         split over pixels with f32 atomics
grad_b (+)= the pixel sums of err, from the same launch (ones operand)
err_input = dgrad(err, W) [* f'(below.output)]  stride 1: the halo conv
                         (conv_hc.hip, conv_hc32 / conv_hc); else the
                         implicit transposed-conv GEMM

When the forward layer runs in fp8 both GEMMs take the e5m2 copy of err:
backward-data against the e4m3 weights, the weight gradient against the
layer's e4m3 input copy (fp8 MFMA kernels; the bias gradient from the same
launch, as the pixel sums of the e5m2 err).  ``root.common.engine.fp8_wgrad = False``
keeps the weight gradient on the bf16 kernel.
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
        # fused gradient quantisation: the GD that produces err_output wrote
        # dy8_ this pass
        self.dy8_fresh_ = False
        self.q8_consumer_ = None

    def __getstate__(self):
        fp8.save_scalers(self, ("fp8_sdy_",))
        return super().__getstate__()

    def fp8_grad_consumer(self):
        return fp8_grad_consumer(self)

    def _q8_target(self, ei):
        return fp8_grad_target(self, ei)

    def run(self):
        fwd = self.forward
        fwd.ensure_params()
        err = self.err_output_effective()
        x = input_tensor(self.input)
        s2d = isinstance(x, ops.S2DImage)   # loader-made s2d input
        squeeze = not s2d and x.dim() == 3
        if squeeze:
            x = x.unsqueeze(-1)
        tmp = ()
        if not s2d and x.dtype != err.dtype:
            x = x.to(err.dtype)
            tmp = (x,)
        pw, pb = fwd._pw_, fwd._pb_
        if self.store_.overwrite and not all(
                self.store_.cleared_by_update(p) for p in (pw, pb)
                if p is not None):
            # the split-K atomics of this layer start from its own zeroed
            # span (normally the update already cleared it: zero_tail)
            self.store_.zero_grads((pw, pb))
        use8 = getattr(fwd, "fp8_", False)
        if use8:
            if self.fp8_sdy_ is None:
                self.fp8_sdy_ = fp8.Scaler(self.torch_device, fp8.E5M2)
                fp8.restore_scaler(self, "fp8_sdy_")
            # the e5m2 copy comes from the epilogue of the GD that produced
            # err_output when it wrote it this pass
            if not self.dy8_fresh_ or self.dy8_ is None or \
                    tuple(self.dy8_.shape) != tuple(err.shape):
                self.dy8_ = fp8.quantize(err, self.fp8_sdy_, out=self.dy8_)
            self.dy8_fresh_ = False
        def wgrad():
            if use8 and self._fp8_wgrad_ok(fwd, x):
                fp8.conv_wgrad(fwd.x8_, fwd.fp8_sx_, self.dy8_,
                               self.fp8_sdy_, pw.grad, fwd.sliding,
                               fwd.padding, fwd.grouping,
                               dbias=None if pb is None else pb.grad)
            else:
                # weight AND bias gradients from one implicit-GEMM launch
                ops.conv_wgrad(x, err, pw.grad, fwd.sliding, fwd.padding,
                               fwd.grouping, col=getattr(fwd, "col_", None),
                               dbias=None if pb is None else pb.grad)

        if self._wgrad_on_side(err):
            # the weight gradient on a branch stream: it runs under this
            # layer's backward-data and the layers below it (LRN / pooling
            # backward, the next backward-data) instead of before them;
            # the parameter store's consumers wait for the stream
            _side_stream_run(self, wgrad, keep=tmp)
        else:
            wgrad()
        if self.need_err_input:
            ei = self.alloc_err_input(tuple(x.shape))
            aux, aux_act = self.aux_tensor()
            if aux is not None and aux.dim() == 3:
                aux = aux.unsqueeze(-1)
            if use8:
                # e5m2 gradient x e4m3 weights on the fp8 MFMA kernel
                wt8 = fp8.permute_for_dgrad(fwd.w8_, fwd.grouping) \
                    if err.is_cuda else None
                q8, qs = self._q8_target(ei)
                fp8.conv_dgrad(self.dy8_, self.fp8_sdy_, fwd.w8_,
                               fwd.fp8_sw_, tuple(x.shape), fwd.sliding,
                               fwd.padding, fwd.grouping, aux=aux,
                               aux_act=aux_act, out=ei, wt8=wt8, q8=q8,
                               q8_scaler=qs)
                if q8 is not None:
                    self.fp8_grad_consumer().dy8_fresh_ = True
            else:
                ops.conv_dgrad(err, fwd.weights_lp, tuple(x.shape),
                               fwd.sliding, fwd.padding, fwd.grouping,
                               aux=aux, aux_act=aux_act, out=ei)
            if squeeze:
                self.err_input.devmem = ei.squeeze(-1)
        self.report_gradients()


    def _wgrad_on_side(self, err):
        return _wgrad_on_side(self, err)

    @staticmethod
    def _fp8_wgrad_ok(fwd, x):
        """the fp8 weight gradient needs the forward's e4m3 input copy of
        this very input (not the s2d / im2col paths)"""
        from veles_amd.utils.config import root, get
        x8 = getattr(fwd, "x8_", None)
        return get(root.common.engine.fp8_wgrad, True) and x8 is not None \
            and not isinstance(x, ops.S2DImage) and \
            tuple(x8.shape) == tuple(x.shape) and x8.device == x.device


class GDTanhConv(GradientDescentConv):
    MAPPING = "conv_tanh"


class GDRELUConv(GradientDescentConv):
    MAPPING = "conv_relu"


class GDStrictRELUConv(GradientDescentConv):
    MAPPING = "conv_str"


class GDSigmoidConv(GradientDescentConv):
    MAPPING = "conv_sigmoid"


# below this many multiply-adds a weight gradient stays on the compute
# stream: a fork / join costs more than the overlap gains at small steps
# (LeNet / CIFAR quick b100: 264-273k / 307-312k samples/s with branch
# streams, 296k / 352k without, profiles/r5/ab_small_wgrad_stream_r5u.log);
# every AlexNet / VGG-16 layer at the bench batches is far above it
_SIDE_MIN_MACS = 1 << 30


def _wgrad_on_side(unit, err):
    """Weight gradients (conv and fully-connected GD units) off the compute
    stream (engine.wgrad_stream / VELES_AMD_WGRAD_STREAM, on by default
    for layers of at least _SIDE_MIN_MACS multiply-adds, except under an
    eager multi-rank backward:
    AlexNet b2048 172.7-173.6k -> 175.0-175.3k img/s on one box with the
    conv ones, profiles/r5/bench_wgrad_stream_ab.md).  Multi-rank, a
    layer's bucket collective waits for it (it is launched from the compute
    stream after the layer's backward-data), so there it overlaps that
    backward-data only."""
    import os
    from veles_amd.utils.config import root, get
    store = getattr(unit, "store_", None)
    env = os.environ.get("VELES_AMD_WGRAD_STREAM")
    if not err.is_cuda or store is None or env == "0" or (
            env is None and not get(root.common.engine.wgrad_stream, True)):
        return False
    if env is None and store._multi() and not store.graph_safe():
        # an eager multi-rank backward (the N > 1 default): the serial weight
        # gradients measured faster there - one-rank RCCL group, AlexNet
        # b2048: 173.6-173.8k img/s against 167.2-168.6k with the branch
        # streams (profiles/r5/ab_solo_eager_wgrad_r5s.log); "1" forces them
        return False
    pw = getattr(getattr(unit, "forward", None), "_pw_", None)
    if env is None and pw is not None and err.dim() > 0 and \
            err.numel() // max(err.shape[-1], 1) * pw.size < _SIDE_MIN_MACS:
        # (output rows) x (weights): the layer's weight-gradient MACs
        return False
    return True


def _side_stream_run(unit, fn, keep=()):
    """Run fn on a branch stream forked from the current one (units.
    _Branches: its scratch buffers are the branch's own, and the scheduler
    / HIP-graph capture joins it at the end); the unit's parameter store is
    told, so that the update waits for the device's branch streams.
    ``keep``:
    temporaries made on the compute stream that fn reads (their memory
    must not be reused before the branch is done with it)."""
    import torch
    from veles_amd.units import _Branches
    (br,) = _Branches.fork(torch.cuda.current_stream().device, 1)
    st = br[0]
    unit.store_.branch_grads = True
    for t in keep:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            t.record_stream(st)
    prev = _Branches._tls.__dict__.get("br")
    _Branches._tls.br = br
    try:
        with torch.cuda.stream(st):
            fn()
    finally:
        _Branches._tls.br = prev


def fp8_grad_consumer(unit):
    """The conv GD whose err_output is ``unit``'s err_input and which runs
    fp8 backward-data on it unmodified (its activation derivative already
    fused into ``unit``'s kernel), or None: ``unit`` then also writes that
    GD's e5m2 gradient copy (fused quantisation)."""
    c = getattr(unit, "q8_consumer_", None)
    if c is None:
        c = False
        for u in getattr(unit, "links_to", ()):
            if isinstance(u, GradientDescentConv) and \
                    getattr(u, "err_output", None) is unit.err_input and \
                    u.need_err_input and getattr(u.forward, "fp8_", False):
                if not (u.own_derivative and
                        getattr(u.forward, "activation", 0)):
                    c = u
                break
        unit.q8_consumer_ = c
    return c or None


def fp8_grad_target(unit, ei):
    """(dy8 buffer, scaler) for ``unit``'s fused gradient quantisation, or
    (None, None) (see conv.fp8_input_target); the caller sets the
    consumer's ``dy8_fresh_``."""
    from veles_amd.utils.config import root, get
    if not get(root.common.engine.fp8_fuse_quant, True):
        return None, None
    c = fp8_grad_consumer(unit)
    if c is None or c.fp8_sdy_ is None or not c.fp8_sdy_.primed or \
            c.dy8_ is None or tuple(c.dy8_.shape) != tuple(ei.shape) or \
            c.dy8_.device != ei.device:
        return None, None
    return c.dy8_, c.fp8_sdy_
