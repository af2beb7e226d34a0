"""Neural-network unit bases (the reconstructed Znicz core).

The Znicz library is absent from the reference snapshot; its API
is rebuilt from the documentation (docs/source/manualrst_veles_workflow_
parameters.rst:465-578, manualrst_veles_workflow_creation.rst:103-145) and
pinned in docs/OPS.md:

* ``Forward`` units own ``weights`` / ``bias`` and map ``input`` -> ``output``;
  weight init ``weights_filling`` in {uniform, gaussian, constant} with
  ``weights_stddev`` (same for bias), ``include_bias``, ``weights_transposed``.
* ``GradientDescentBase`` units map ``err_output`` -> ``err_input`` and produce
  the parameter gradients; hyper-parameters ``learning_rate[_bias]``,
  ``weights_decay[_bias]``, ``l1_vs_l2[_bias]``, ``gradient_moment[_bias]``,
  ``accumulate_gradient``, ``need_err_input``.

MI355X execution: parameters live in the workflow's flat ParameterStore
(veles_amd/models/params.py); every GD unit enqueues its gradient kernels and
reports readiness; the store launches the bucketed RCCL all-reduce and, after
the last GD unit, ONE fused SGD kernel.  The activation derivative of layer
L is folded into the err_input epilogue of the unit above it whenever that
unit's kernel supports it (``aux`` multiply), saving a full read/write pass.
"""
from __future__ import annotations

import numpy

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.prng import random_generator
from veles_amd import ops

__all__ = ["Forward", "GradientDescentBase", "fill_weights",
           "get_param_store", "ACTIVATION_MODES"]

ACTIVATION_MODES = {0: "ACTIVATION_LINEAR", 1: "ACTIVATION_TANH",
                    2: "ACTIVATION_RELU", 3: "ACTIVATION_STRICT_RELU",
                    4: "ACTIVATION_SIGMOID"}


def fill_weights(arr, filling, stddev, prng):
    if filling == "uniform":
        prng.fill(arr, -stddev, stddev)
    elif filling == "gaussian":
        prng.fill_normal_real(arr, 0.0, stddev)
    elif filling == "constant":
        arr[...] = stddev
    else:
        raise ValueError("Unknown weights filling %r" % filling)


def get_param_store(unit):
    """The flat parameter store of the unit's workflow for its device."""
    from veles_amd.models.params import ParameterStore
    wf = unit.workflow
    store = getattr(wf, "param_store_", None)
    if store is None or store.device is not unit.device:
        from veles_amd.parallel import find_dp
        store = ParameterStore(unit.device, find_dp(wf))
        wf.param_store_ = store
    return store



def _sync_device(t):
    """Wait for ALL streams of ``t``'s device before a host read for a
    snapshot: the update may have run on the compute stream of the
    workflow (or inside a replayed HIP graph launched there) or on the
    update side stream, and ``Tensor.cpu()`` orders only against the
    CURRENT stream, which outside a workflow run is another one."""
    if t is not None and getattr(t, "is_cuda", False):
        import torch
        torch.cuda.synchronize(t.device)

class Forward(AcceleratedUnit):
    """Base forward layer."""
    hide_from_registry = True
    ACTIVATION = 0
    has_weights = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.weights_filling = kwargs.get("weights_filling", "uniform")
        self.weights_stddev = kwargs.get("weights_stddev", None)
        self.bias_filling = kwargs.get("bias_filling", "uniform")
        self.bias_stddev = kwargs.get("bias_stddev", None)
        self.include_bias = kwargs.get("include_bias", True)
        self.weights_transposed = kwargs.get("weights_transposed", False)
        self.rand = kwargs.get("rand", random_generator.get())
        self.weights = Array()
        self.bias = Array()
        self.output = Array(shallow_pickle=True)
        self.demand("input")

    def init_unpickled(self):
        super().init_unpickled()
        self._pw_ = None
        self._pb_ = None

    @property
    def activation(self):
        return self.ACTIVATION

    @property
    def activation_mode(self):
        return ACTIVATION_MODES.get(self.activation, "ACTIVATION_LINEAR")

    # parameter plumbing ----------------------------------------------------
    def register_params(self, wshape, fan_in):
        """Create (or restore) weights/bias on the host and register them in
        the flat store."""
        if self.weights.mem is None or self.weights.mem.shape != tuple(wshape):
            w = numpy.zeros(wshape, numpy.float32)
            std = self.weights_stddev
            if std is None:
                std = 1.0 / numpy.sqrt(max(fan_in, 1))
            fill_weights(w, self.weights_filling, std, self.rand)
            self.weights.reset(w)
        if self.include_bias:
            n = wshape[0]
            if self.bias.mem is None or self.bias.mem.shape != (n,):
                b = numpy.zeros(n, numpy.float32)
                std = self.bias_stddev
                if std is None:
                    std = 1.0 / numpy.sqrt(max(fan_in, 1))
                fill_weights(b, self.bias_filling, std, self.rand)
                self.bias.reset(b)
        store = get_param_store(self)
        self._pw_ = store.register(self, "weights", self.weights.mem)
        self._pb_ = store.register(self, "bias", self.bias.mem) \
            if self.include_bias else None
        self.store_ = store

    def ensure_params(self):
        st = self.store_
        if not st.finalized:
            st.finalize()

    @property
    def weights_lp(self):
        """Compute-dtype weights (bf16 view on the GPU)."""
        self.ensure_params()
        return self._pw_.lp

    @property
    def weights_master(self):
        self.ensure_params()
        return self._pw_.master

    @property
    def bias_master(self):
        if self._pb_ is None:
            return None
        self.ensure_params()
        return self._pb_.master

    def sync_params_to_host(self):
        _sync_device(getattr(self._pw_, "master", None))
        if self._pw_ is not None and self._pw_.master is not None:
            self.weights.reset(self._pw_.master.detach().float().cpu().numpy()
                               .reshape(self.weights.mem.shape))
            self._pw_.host = self.weights.mem
            if self._pb_ is not None and self._pb_.master is not None:
                self.bias.reset(self._pb_.master.detach().float().cpu()
                                .numpy())
                self._pb_.host = self.bias.mem

    def __getstate__(self):
        self.sync_params_to_host()
        return super().__getstate__()

    def alloc_output(self, shape, dtype=None):
        import torch
        dt = dtype or self.compute_dtype
        t = self.output.devmem
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dt or \
                t.device != self.torch_device:
            self.output.devmem = torch.zeros(shape, dtype=dt,
                                             device=self.torch_device)
        return self.output.devmem

    def input_tensor(self, dtype=None):
        t = self.input.devmem
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        return t

    def package_export(self):
        self.sync_params_to_host()
        d = {"weights": self.weights.mem, "include_bias": self.include_bias,
             "weights_transposed": self.weights_transposed,
             "activation_mode": self.activation_mode}
        if self.include_bias:
            d["bias"] = self.bias.mem
        return d


class GradientDescentBase(AcceleratedUnit):
    """Base backward layer."""
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "TRAINER")
        super().__init__(workflow, **kwargs)
        self.learning_rate = kwargs.get("learning_rate", 0.01)
        self.learning_rate_bias = kwargs.get("learning_rate_bias",
                                             self.learning_rate)
        self.weights_decay = kwargs.get("weights_decay", 0.0)
        self.weights_decay_bias = kwargs.get("weights_decay_bias", 0.0)
        self.l1_vs_l2 = kwargs.get("l1_vs_l2", 0.0)
        self.l1_vs_l2_bias = kwargs.get("l1_vs_l2_bias", self.l1_vs_l2)
        self.gradient_moment = kwargs.get("gradient_moment", 0.0)
        self.gradient_moment_bias = kwargs.get("gradient_moment_bias",
                                               self.gradient_moment)
        self.accumulate_gradient = kwargs.get("accumulate_gradient", False)
        # adaptive solvers (one of momentum / adagrad / adadelta per unit)
        solvers = kwargs.get("solvers", ("momentum",))
        if isinstance(solvers, str):
            solvers = (solvers,)
        self.solvers = set(solvers)
        unknown = self.solvers - set(ops.SOLVERS) - {"fast"}
        if unknown:
            raise ValueError("Unknown solvers %s" % sorted(unknown))
        self.adagrad_epsilon = kwargs.get("adagrad_epsilon", 1e-8)
        self.adadelta_momentum = kwargs.get("adadelta_momentum", 0.9)
        self.adadelta_epsilon = kwargs.get("adadelta_epsilon", 1e-8)
        self.adadelta_adom = kwargs.get("adadelta_adom", 0.3)
        self.fast_learning_rate = kwargs.get("fast_learning_rate", 0.02)
        self.factor_ortho = kwargs.get("factor_ortho", 0)
        self.variant_gradient = kwargs.get("variant_gradient", True)
        self.variant_moment_gradient = kwargs.get(
            "variant_moment_gradient", True)
        self.last_minibatch = kwargs.get("last_minibatch", False)
        self.need_err_input = kwargs.get("need_err_input", True)
        self.apply_gradient = kwargs.get("apply_gradient", True)
        self.err_input = Array(shallow_pickle=True)
        self.accumulated_gradient_weights = Array()
        self.accumulated_gradient_bias = Array()
        # activation derivative handling (see module docstring)
        self.own_derivative = True       # apply f'(output) to err_output
        self.fused_aux = None            # unit whose output is the aux
        self.fused_aux_act = 0
        self.demand("err_output", "input")

    def init_unpickled(self):
        super().init_unpickled()
        self.tmp_err_ = None

    def hyper(self, is_bias):
        if not self.apply_gradient:
            return 0.0, 0.0, 0.0, 0.0
        if is_bias:
            return (self.learning_rate_bias, self.weights_decay_bias,
                    self.l1_vs_l2_bias, self.gradient_moment_bias)
        return (self.learning_rate, self.weights_decay, self.l1_vs_l2,
                self.gradient_moment)

    SOLVER = None  # a subclass may force one (RPropAll2All: "rprop")

    def solver(self):
        """(mode, eps, rho) of this unit's update rule (ops.SOLVERS)."""
        names = getattr(self, "solvers", ("momentum",))
        if self.SOLVER is not None:
            return ops.SOLVERS[self.SOLVER], 0.0, 0.0
        if "adadelta" in names:
            return (ops.SOLVERS["adadelta"], self.adadelta_epsilon,
                    self.adadelta_momentum)
        if "adagrad" in names:
            return ops.SOLVERS["adagrad"], self.adagrad_epsilon, 0.0
        return 0, 0.0, 0.0

    @property
    def forward(self):
        return getattr(self, "forward_unit", None)

    def attach_params(self, fwd):
        """Bind this GD unit to the forward unit's parameters in the store."""
        self.forward_unit = fwd
        store = fwd.store_
        self.store_ = store
        self.params_ = []
        for p in (fwd._pw_, fwd._pb_):
            if p is not None:
                store.attach_gd(p, self)
                self.params_.append(p)
        for arr, p in ((self.accumulated_gradient_weights, fwd._pw_),
                       (self.accumulated_gradient_bias, fwd._pb_)):
            mom = arr.mem
            if mom is not None and p is not None and mom.shape == p.shape:
                p.host_mom = mom

    def fuse_from(self, producer_unit, act):
        """This unit's err_input will be multiplied by f'(producer.output)
        (the activation of the layer below)."""
        self.fused_aux = producer_unit
        self.fused_aux_act = act

    def aux_tensor(self):
        if self.fused_aux is None or not self.fused_aux_act:
            return None, 0
        return self.fused_aux.output.devmem, self.fused_aux_act

    def err_output_effective(self):
        """err_output with this layer's activation derivative applied (when
        not already fused into the producer of err_output)."""
        fwd = self.forward
        err = self.err_output.devmem
        act = getattr(fwd, "activation", 0) if fwd is not None else 0
        if not self.own_derivative or not act:
            return err
        if self.tmp_err_ is None or self.tmp_err_.shape != err.shape or \
                self.tmp_err_.dtype != err.dtype:
            import torch
            self.tmp_err_ = torch.empty_like(err)
        return ops.act_bwd(err, fwd.output.devmem, act, out=self.tmp_err_)

    def alloc_err_input(self, shape, dtype=None):
        import torch
        dt = dtype or self.compute_dtype
        t = self.err_input.devmem
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dt or \
                t.device != self.torch_device:
            self.err_input.devmem = torch.zeros(shape, dtype=dt,
                                                device=self.torch_device)
        return self.err_input.devmem

    def report_gradients(self):
        store = self.store_
        store.grads_ready(self.params_)
        if store.all_ready():
            store.apply()

    def __getstate__(self):
        fwd = getattr(self, "forward_unit", None)
        pw = getattr(fwd, "_pw_", None)  # parameterless layers: pooling...
        _sync_device(getattr(pw, "mom", None))
        if pw is not None and pw.mom is not None:
            self.accumulated_gradient_weights.reset(
                pw.mom.detach().float().cpu().numpy())
            if getattr(fwd, "_pb_", None) is not None:
                self.accumulated_gradient_bias.reset(
                    fwd._pb_.mom.detach().float().cpu().numpy())
        return super().__getstate__()
