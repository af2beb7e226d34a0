"""StandardWorkflow: a full training loop assembled from a ``layers`` list.

Reference API (documented; the Znicz source is absent):
docs/source/manualrst_veles_workflow_creation.rst:103-470 (``link_*``
builders, canonical cycle :117-143), manualrst_veles_workflow_parameters.rst
(layer types :465-500, ``->`` / ``<-`` kwargs :506-578, ``mcdnnic_topology``
:580-599, decision / snapshotter / lr_adjuster keys).

Canonical cycle::

    repeater <- start_point ; loader <- repeater ; forwards <- loader
    evaluator <- forwards[-1] ; decision <- evaluator
    snapshotter <- decision ; gds (reverse) <- snapshotter
    repeater <- gds[0] ; end_point <- snapshotter (gated by decision.complete)

GD units are gate-skipped on non-TRAIN minibatches (``decision.gd_skip``) and
blocked once training completes.  The activation derivative of layer i-1
is fused into gds[i]'s err_input kernel (see models/nn_units.py).
"""
from __future__ import annotations

import os
import re

from veles_amd.accelerated_units import AcceleratedWorkflow
from veles_amd.loader.base import UserLoaderRegistry
from veles_amd.models import activation as act_units
from veles_amd.models.all2all import (
    All2All, All2AllRELU, All2AllSigmoid, All2AllSoftmax, All2AllStrictRELU,
    All2AllTanh, ResizableAll2All)
from veles_amd.models.conv import (
    Conv, ConvRELU, ConvSigmoid, ConvStrictRELU, ConvTanh)
from veles_amd.models.decision import DecisionGD, DecisionMSE
from veles_amd.models.dropout import DropoutBackward, DropoutForward
from veles_amd.models.evaluator import EvaluatorMSE, EvaluatorSoftmax
from veles_amd.models.gd import (
    GDRELU, GDSigmoid, GDSoftmax, GDStrictRELU, GDTanh, GradientDescent)
from veles_amd.models.gd_conv import (
    GDRELUConv, GDSigmoidConv, GDStrictRELUConv, GDTanhConv,
    GradientDescentConv)
from veles_amd.models.lr_adjust import LearningRateAdjust
from veles_amd.models.normalization_units import (
    LRNormalizerBackward, LRNormalizerForward)
from veles_amd.models.pooling import (
    AvgPooling, Depooling, GDAvgPooling, GDDepooling, GDMaxAbsPooling,
    GDMaxPooling, GDPoolDepool, MaxAbsPooling, MaxPooling,
    StochasticAbsPooling, StochasticAbsPoolingDepooling, StochasticPooling,
    StochasticPoolingDepooling)
from veles_amd.models.channel_splitting import (
    ChannelMerger, ChannelSplitter, GDChannelMerger, GDChannelSplitter)
from veles_amd.models.cutter import Cutter, GDCutter
from veles_amd.models.deconv import Deconv, GDDeconv
from veles_amd.models.rprop_all2all import RPropAll2All
from veles_amd.models.standard_workflow_links import LinkBuilders
from veles_amd.models.weights_zerofilling import GDZeroFiller, ZeroFiller
from veles_amd.plumbing import Repeater
from veles_amd.snapshotter import SnapshotterRegistry, SnapshotterToFile
from veles_amd.utils.config import Config, fix_contents

__all__ = ["StandardWorkflow", "LAYER_TYPES", "parse_mcdnnic"]

LAYER_TYPES = {
    "all2all": (All2All, GradientDescent),
    "all2all_resizable": (ResizableAll2All, GradientDescent),
    "all2all_tanh": (All2AllTanh, GDTanh),
    "all2all_relu": (All2AllRELU, GDRELU),
    "all2all_str": (All2AllStrictRELU, GDStrictRELU),
    "all2all_sigmoid": (All2AllSigmoid, GDSigmoid),
    "softmax": (All2AllSoftmax, GDSoftmax),
    "conv": (Conv, GradientDescentConv),
    "conv_tanh": (ConvTanh, GDTanhConv),
    "conv_relu": (ConvRELU, GDRELUConv),
    "conv_str": (ConvStrictRELU, GDStrictRELUConv),
    "conv_sigmoid": (ConvSigmoid, GDSigmoidConv),
    "max_pooling": (MaxPooling, GDMaxPooling),
    "avg_pooling": (AvgPooling, GDAvgPooling),
    "maxabs_pooling": (MaxAbsPooling, GDMaxAbsPooling),
    "stochastic_pooling": (StochasticPooling, GDMaxPooling),
    "stochastic_abs_pooling": (StochasticAbsPooling, GDMaxAbsPooling),
    "stochastic_pool_depool": (StochasticPoolingDepooling, GDPoolDepool),
    "stochastic_abs_pool_depool": (StochasticAbsPoolingDepooling,
                                   GDPoolDepool),
    "depooling": (Depooling, GDDepooling),
    "deconv": (Deconv, GDDeconv),
    "cutter": (Cutter, GDCutter),
    "channel_splitter": (ChannelSplitter, GDChannelSplitter),
    "channel_merger": (ChannelMerger, GDChannelMerger),
    "zero_filter": (ZeroFiller, GDZeroFiller),
    "rprop_all2all": (All2All, RPropAll2All),
    "norm": (LRNormalizerForward, LRNormalizerBackward),
    "dropout": (DropoutForward, DropoutBackward),
    "activation_tanh": (act_units.ForwardTanh, act_units.BackwardTanh),
    "activation_relu": (act_units.ForwardRELU, act_units.BackwardRELU),
    "activation_str": (act_units.ForwardStrictRELU,
                       act_units.BackwardStrictRELU),
    "activation_sigmoid": (act_units.ForwardSigmoid,
                           act_units.BackwardSigmoid),
    "activation_log": (act_units.ForwardLog, act_units.BackwardLog),
    "activation_tanhlog": (act_units.ForwardTanhLog,
                           act_units.BackwardTanhLog),
    "activation_sincos": (act_units.ForwardSinCos, act_units.BackwardSinCos),
    "activation_mul": (act_units.ForwardMul, act_units.BackwardMul),
}

# GD classes whose err_input kernel can multiply by f'(aux) in its epilogue
_FUSABLE = (GradientDescent, GradientDescentConv, GDMaxPooling, GDAvgPooling,
            GDMaxAbsPooling, LRNormalizerBackward, DropoutBackward,
            act_units.ActivationBackward)
_POOL_KW = ("kx", "ky", "sliding")
_LRN_KW = ("alpha", "beta", "k", "n")


def parse_mcdnnic(topology, params=None):
    """"12x256x256-32C4-MP2-64C4-MP3-32N-4N" -> layers list (reference docs
    :580-599).  C = conv (strict relu), MP = max pooling, N = fully
    connected (the last one softmax)."""
    params = params or {}
    parts = topology.split("-")
    layers = []
    for i, p in enumerate(parts[1:]):
        last = i == len(parts) - 2
        m = re.match(r"^(\d+)C(\d+)$", p)
        if m:
            layers.append({"type": "conv_str", "->": dict(
                params.get("->", {}), n_kernels=int(m.group(1)),
                kx=int(m.group(2)), ky=int(m.group(2))),
                "<-": dict(params.get("<-", {}))})
            continue
        m = re.match(r"^MP(\d+)$", p)
        if m:
            k = int(m.group(1))
            layers.append({"type": "max_pooling",
                           "->": {"kx": k, "ky": k, "sliding": (k, k)}})
            continue
        m = re.match(r"^(\d+)N$", p)
        if m:
            layers.append({"type": "softmax" if last else "all2all_tanh",
                           "->": dict(params.get("->", {}),
                                      output_sample_shape=int(m.group(1))),
                           "<-": dict(params.get("<-", {}))})
            continue
        raise ValueError("Unknown mcdnnic layer %r" % p)
    return layers


def _cfg(v):
    return fix_contents(v) if isinstance(v, Config) else (v or {})


class StandardWorkflow(LinkBuilders, AcceleratedWorkflow):
    """kwargs: layers | mcdnnic_topology (+mcdnnic_parameters), loader_name,
    loader_config, loss_function ("softmax"|"mse"), decision_config,
    snapshotter_config (None disables), lr_adjuster_config, evaluator_config,
    testing; configs of the optional builders (standard_workflow_links.py):
    image_saver_config, data_saver_config, publisher_config,
    result_unit_config."""

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        layers = _cfg(kwargs.get("layers"))
        if not layers and kwargs.get("mcdnnic_topology"):
            layers = parse_mcdnnic(kwargs["mcdnnic_topology"],
                                   _cfg(kwargs.get("mcdnnic_parameters")))
        self.layers = list(layers or [])
        self.loader_name = kwargs.get("loader_name")
        self.loader_config = dict(_cfg(kwargs.get("loader_config")))
        self.loss_function = kwargs.get("loss_function", "softmax")
        # LRN -> 3x3 max pooling pairs as one fused kernel each way
        self.fuse_lrn_pool = kwargs.get("fuse_lrn_pool", True)
        self.decision_config = dict(_cfg(kwargs.get("decision_config")))
        self.snapshotter_config = kwargs.get("snapshotter_config")
        if self.snapshotter_config is not None:
            self.snapshotter_config = dict(_cfg(self.snapshotter_config))
        self.lr_adjuster_config = kwargs.get("lr_adjuster_config")
        self.evaluator_config = dict(_cfg(kwargs.get("evaluator_config")))
        self.testing = kwargs.get("testing", False)
        # eager passes per (class, batch size) before a segment is captured
        self.graph_warmup = int(kwargs.get("graph_warmup", 2))
        for k in ("image_saver_config", "data_saver_config",
                  "publisher_config", "result_unit_config"):
            setattr(self, k, dict(_cfg(kwargs.get(k))))
        self.forwards = []
        self.gds = []
        self.snapshotter = None
        self.lr_adjuster = None
        self.create_workflow()

    # -- builders (names follow the documented link_* API) ----------------
    def create_workflow(self):
        self.link_repeater(self.start_point)
        self.link_loader(self.repeater)
        last = self.link_forwards(("input", "minibatch_data"), self.loader)
        last = self.link_evaluator(last)
        last = self.link_decision(last)
        if self.snapshotter_config is not None and not self.testing:
            last = self.link_snapshotter(last)
        if not self.testing:
            last_gd = self.link_gds(last)
            if self.lr_adjuster_config:
                last_gd = self.link_lr_adjuster(last_gd)
            self.link_loop(last_gd)
        else:
            last = self.link_output_collector(last)
            self.link_loop(last)
        self.link_end_point(last)

    def link_output_collector(self, *parents):
        from veles_amd.models.result_collector import OutputCollector
        self.output_collector = OutputCollector(self)
        self.output_collector.link_from(*parents)
        self.output_collector.link_attrs(self.forwards[-1], "output")
        self.output_collector.link_attrs(
            self.loader, "minibatch_class", "minibatch_size",
            "minibatch_indices")
        self.output_collector.labels_source = self.loader
        return self.output_collector

    def switch_to_testing(self):
        """Turn a trained (e.g. snapshot-restored) workflow into a test run
        (``--test -w snapshot``): serve the TEST class once, no backward, no
        snapshots, collect ``Output`` / ``Labels`` into the results."""
        from veles_amd.mutable import Bool
        self.testing = True
        self.loader.testing = True
        for gd in self.gds:
            gd.gate_block = Bool(True)
        if self.lr_adjuster is not None:
            self.lr_adjuster.gate_block = Bool(True)
        if self.snapshotter is not None:
            self.snapshotter.gate_block = Bool(True)
        if getattr(self, "output_collector", None) is None:
            self.link_output_collector(self.decision)
            self.repeater.unlink_from(self.gds[0] if self.gds else
                                      self.decision)
            self.repeater.link_from(self.output_collector)
            # finish only after the last test minibatch was collected
            for u in list(self.end_point.links_from):
                self.end_point.unlink_from(u)
            self.end_point.link_from(self.output_collector)
        d = self.decision
        d.max_epochs = d.epoch_number + 1
        d.fail_iterations = None
        d.complete <<= False
    def link_repeater(self, *parents):
        self.repeater = Repeater(self)
        self.repeater.link_from(*parents)
        return self.repeater

    def link_loader(self, *parents):
        cls = UserLoaderRegistry.loaders.get(self.loader_name)
        if cls is None:
            raise ValueError("Unknown loader %r (known: %s)" % (
                self.loader_name, sorted(UserLoaderRegistry.loaders)))
        cfg = dict(self.loader_config)
        if self.testing:
            cfg["testing"] = True
        self.loader = cls(self, **cfg)
        self.loader.link_from(*parents)
        return self.loader

    def _split_kwargs(self, layer):
        fwd = dict(layer.get("->", {}))
        bwd = dict(layer.get("<-", {}))
        for k, v in layer.items():
            if k in ("type", "->", "<-", "name"):
                continue
            fwd.setdefault(k, v)
            bwd.setdefault(k, v)
        return fwd, bwd

    def link_forwards(self, init_attrs, *parents):
        prev = None
        pools, convs, weighted = [], [], None
        for i, layer in enumerate(self.layers):
            typ = layer["type"]
            fcls, _ = LAYER_TYPES[typ]
            fwd_kw, _ = self._split_kwargs(layer)
            allowed = getattr(fcls, "KNOWN_KWARGS", None)
            name = layer.get("name", "%s%d" % (typ, i))
            unit = fcls(self, name=name, **self._filter(fcls, fwd_kw))
            if prev is None:
                unit.link_from(*parents)
                unit.link_attrs(parents[0], init_attrs)
            else:
                unit.link_from(prev)
                unit.link_attrs(prev, ("input", "output"))
            if isinstance(unit, DropoutForward):
                unit.link_attrs(self.loader, "minibatch_class")
            # encoder/decoder pairing (auto-encoders): depooling inverts the
            # latest pooling, deconv the latest conv (LIFO)
            if isinstance(unit, Depooling):
                if not pools:
                    raise ValueError("depooling without a pooling before it")
                pool = pools.pop()
                unit.link_attrs(pool, "input_offset")
                pool.offsets_exported = True  # keep int32 flat offsets
                unit.output_shape_source = pool.input
                unit.geometry = (pool.ky, pool.kx, tuple(pool.sliding))
            elif isinstance(unit, (MaxPooling, MaxAbsPooling,
                                   StochasticPooling)) and \
                    not isinstance(unit, StochasticPoolingDepooling):
                pools.append(unit)
            if isinstance(unit, Deconv):
                if unit.output_shape_source is None and \
                        unit.n_channels is None and convs:
                    unit.output_shape_source = convs.pop()
            elif isinstance(unit, Conv):
                convs.append(unit)
            if isinstance(unit, ZeroFiller) and unit.weights_unit is None:
                unit.weights_unit = weighted
            if getattr(unit, "has_weights", False) and \
                    hasattr(unit, "register_params"):
                weighted = unit
            self.forwards.append(unit)
            prev = unit
            del allowed
        return prev

    @staticmethod
    def _filter(cls, kw):
        known = cls.known_kwargs()
        base = {"name", "view_group", "ignore_gate", "timings", "force_cpu"}
        out = {}
        for k, v in kw.items():
            if k in known or k in base:
                out[k] = v
        return out

    def link_evaluator(self, *parents):
        last = self.forwards[-1]
        if self.loss_function == "softmax":
            self.evaluator = EvaluatorSoftmax(self, **self.evaluator_config)
            self.evaluator.link_attrs(last, "output")
            if isinstance(last, All2AllSoftmax):
                self.evaluator.logits = last.logits
            self.evaluator.link_attrs(self.loader,
                                      ("labels", "minibatch_labels"))
        else:
            self.evaluator = EvaluatorMSE(self, **self.evaluator_config)
            self.evaluator.link_attrs(last, "output")
            self.evaluator.link_attrs(self.loader,
                                      ("target", "minibatch_targets"))
        self.evaluator.link_attrs(
            self.loader, ("batch_size", "minibatch_size"),
            ("global_batch_size", "global_minibatch_size"), "minibatch_class")
        self.evaluator.link_from(*parents)
        return self.evaluator

    def link_decision(self, *parents):
        cls = DecisionGD if self.loss_function == "softmax" else DecisionMSE
        self.decision = cls(self, **self.decision_config)
        self.decision.link_from(*parents)
        self.decision.link_attrs(self.loader, "minibatch_class",
                                 "last_minibatch", "class_lengths",
                                 "epoch_ended", "minibatch_size")
        self.decision.link_attrs(self.loader, "epoch_number", two_way=True)
        self.decision.evaluator = self.evaluator
        return self.decision

    def link_snapshotter(self, *parents):
        cfg = dict(self.snapshotter_config)
        kind = cfg.pop("kind", "file")
        cls = SnapshotterRegistry.snapshotters.get(kind, SnapshotterToFile)
        self.snapshotter = cls(self, **cfg)
        self.snapshotter.link_from(*parents)
        self.snapshotter.link_attrs(self.decision,
                                    ("suffix", "snapshot_suffix"))
        self.snapshotter.gate_skip = ~self.decision.epoch_ended_flag | \
            ~self.decision.improved
        return self.snapshotter

    def link_gds(self, *parents):
        n = len(self.forwards)
        gds = [None] * n
        prev = None
        for i in reversed(range(n)):
            layer = self.layers[i]
            _, gcls = LAYER_TYPES[layer["type"]]
            fwd = self.forwards[i]
            _, bwd_kw = self._split_kwargs(layer)
            kw = self._filter(gcls, bwd_kw)
            if isinstance(fwd, (MaxPooling, AvgPooling, MaxAbsPooling,
                                StochasticPooling)):
                kw.update(kx=fwd.kx, ky=fwd.ky, sliding=fwd.sliding)
            if isinstance(fwd, LRNormalizerForward):
                kw.update(alpha=fwd.alpha, beta=fwd.beta, k=fwd.k, n=fwd.n)
            gd = gcls(self, name="gd_" + fwd.name, **kw)
            gd.forward_unit = fwd
            gd.link_attrs(fwd, "input")
            if hasattr(fwd, "output"):
                gd.link_attrs(fwd, "output")
            if hasattr(fwd, "input_offset") and "input_offset" in gd.demanded:
                gd.link_attrs(fwd, "input_offset")
            if isinstance(fwd, act_units.ActivationForward):
                gd.factor = getattr(fwd, "factor", 1.0)
            if prev is None:
                gd.link_attrs(self.evaluator, "err_output")
                gd.link_from(*parents)
            else:
                gd.link_attrs(prev, ("err_output", "err_input"))
                gd.link_from(prev)
            gd.gate_block = self.decision.complete
            gd.gate_skip = self.decision.gd_skip
            gds[i] = gd
            prev = gd
        gds[0].need_err_input = False
        # fold the activation derivative of layer i-1 into gds[i]
        for i in range(1, n):
            below = self.forwards[i - 1]
            act = getattr(below, "activation", 0)
            if act and isinstance(gds[i], _FUSABLE) and \
                    getattr(gds[i - 1], "own_derivative", False):
                gds[i].fuse_from(below, act)
                gds[i - 1].own_derivative = False
        # LRN -> max pooling pairs run as one fused kernel each way
        for i in range(n - 1):
            lrn, pool = self.forwards[i], self.forwards[i + 1]
            if isinstance(lrn, LRNormalizerForward) and \
                    type(pool) is MaxPooling and self.fuse_lrn_pool:
                lrn.fused_into = pool
                pool.fused_lrn = lrn
                gds[i + 1].fused_lrn_gd = gds[i]
        self.gds = gds
        return gds[0]

    def link_lr_adjuster(self, *parents):
        cfg = dict(_cfg(self.lr_adjuster_config))
        self.lr_adjuster = LearningRateAdjust(self, **cfg)
        for gd in self.gds:
            if hasattr(gd, "params_") or isinstance(
                    gd, (GradientDescent, GradientDescentConv)):
                self.lr_adjuster.add_gd_unit(gd)
        self.lr_adjuster.link_attrs(self.loader, "minibatch_class")
        self.lr_adjuster.link_from(*parents)
        self.lr_adjuster.gate_block = self.decision.complete
        return self.lr_adjuster

    def link_loop(self, *parents):
        self.repeater.link_from(*parents)
        self.repeater.gate_block = self.decision.complete | \
            self.decision.steps_complete

    def link_end_point(self, *parents):
        self.end_point.link_from(*parents)
        self.end_point.gate_block = ~self.decision.complete

    # -- execution helpers ------------------------------------------------
    def initialize(self, **kwargs):
        self.param_store_ = None
        from veles_amd.parallel import find_dp
        dp = find_dp(self)
        if dp is not None:
            self.loader.rank = dp.rank
            self.loader.world_size = dp.world_size
        # gradient accumulation (elastic shrink, parallel/launch.py): each
        # micro-step serves 1/acc of the configured global minibatch, the
        # optimizer steps once per acc micro-steps
        from veles_amd.utils.config import root, get
        acc = max(1, int(get(root.common.engine.dp.accumulate,
                             os.environ.get("VELES_AMD_DP_ACCUMULATE", 1))))
        ld = self.loader
        full = getattr(ld, "full_minibatch_size", None) or \
            ld.max_minibatch_size
        ld.full_minibatch_size = full
        ld.max_minibatch_size = -(-full // acc)
        res = super().initialize(**kwargs)
        # forward / backward HIP-graph segments (GPU only; veles_amd/graphs)
        from veles_amd.graphs import install_step_graphs
        install_step_graphs(self, warmup=self.graph_warmup)
        # a run-ahead loader gathers the next minibatch as the backward
        # starts (FullBatchLoader._defer_runahead)
        gds = [g for g in reversed(getattr(self, "gds", []) or [])
               if g is not None]
        if gds and hasattr(ld, "launch_runahead"):
            ld.runahead_anchor_ = gds[0]
            gds[0].before_run_ = [ld.launch_runahead]
        return res

    def run_steps(self, n):
        """Run exactly ``n`` more TRAIN minibatches (benchmarks / tests)."""
        d = self.decision
        d.max_steps = d.train_steps + n
        d.steps_complete <<= False
        for u in self:
            u.stopped = False
        self.run()

    def extract_forward_workflow(self, loader_name=None, loader_config=None,
                                 result_unit_factory=None,
                                 result_unit_config=None, cyclic=False):
        """A test-mode forward-only workflow sharing the trained layers
        (reference docs manualrst_veles_example_advanced.rst:327-377)."""
        from veles_amd.models.forward_workflow import ForwardWorkflow
        return ForwardWorkflow.from_trained(
            self, loader_name or self.loader_name,
            loader_config if loader_config is not None else
            self.loader_config, result_unit_factory, result_unit_config,
            cyclic)
