"""Optional ``link_*`` builders of StandardWorkflow: normalisation, double
buffering, data / image dumps, the interactive shell, reports, forward
workflow extraction and every plotter of Znicz' StandardWorkflow.

Reference API (documented; the Znicz source is absent):
docs/source/manualrst_veles_workflow_creation.rst:103-640 - ``link_meandispnorm``
(:153-167, rule 12), ``link_avatar`` (rule 6), ``link_image_saver`` (rule 10),
``link_ipython`` (rule 13), ``link_result_unit`` (rule 14),
``link_data_saver`` (rule 15), the error / matrix plotters (rule 16),
``link_immediate_plotter`` / ``link_weights_plotter`` (rule 17),
``link_similar_weights_plotter`` (rule 18), ``link_image_plotter`` (rule 19),
``link_table_plotter`` (rule 20); ``link_publisher`` in the builder list.

Every builder follows the documented convention: it creates ONE unit (or a
chain of plotters), links its data attributes to the units that must already
exist, links its control flow from ``*parents`` and returns the (last) unit,
stored as ``self.<name>``.  Plotters skip every run except the one right
after an epoch ends (``gate_skip = ~decision.epoch_ended_flag``) and render
files on rank 0 only (plotter.py).
"""
from __future__ import annotations

from veles_amd.loader.base import CLASS_NAME, TEST, TRAIN, VALID

__all__ = ["LinkBuilders"]


class LinkBuilders(object):
    """Mixed into StandardWorkflow (models/standard_workflow.py)."""

    # -- helpers ----------------------------------------------------------
    def _require(self, *names):
        for n in names:
            if getattr(self, n, None) is None:
                raise AttributeError(
                    "link the %s unit first (docs: rules for linking units "
                    "in StandardWorkflow)" % n)

    def _epoch_plotter_gate(self, unit):
        unit.gate_skip = ~self.decision.epoch_ended_flag
        return unit

    def _chain(self, units, parents):
        """Link ``units`` one after another from ``parents``."""
        prev = parents
        for u in units:
            u.link_from(*prev)
            prev = (u,)
        return units[-1]

    def _weighted_forwards(self):
        # decided by class (parameters register only at initialize)
        return [f for f in self.forwards
                if getattr(f, "has_weights", False) and
                hasattr(f, "register_params")]

    # -- data path --------------------------------------------------------
    def link_meandispnorm(self, *parents):
        """MeanDispNormalizer between the loader and the first layer:
        ``(minibatch_data - mean) * rdisp`` with the loader's ``mean`` /
        ``rdisp`` (a full-batch loader then serves raw samples instead of
        normalising in its gather: ``export_affine``).  Link the forwards
        with ``("input", "output")`` from ``self.meandispnorm``."""
        from veles_amd.mean_disp_normalizer import MeanDispNormalizer
        self._require("loader")
        self.meandispnorm = MeanDispNormalizer(self)
        self.meandispnorm.link_attrs(self.loader, ("input", "minibatch_data"))
        ld = self.loader
        if getattr(ld, "mean", None) is None or \
                getattr(ld, "rdisp", None) is None:
            raise ValueError("link_meandispnorm: %s exports no mean / rdisp"
                             % type(ld).__name__)
        # the loader serves raw samples and publishes its normalisation
        if hasattr(ld, "export_affine"):
            ld.export_affine = True
        self.meandispnorm.link_attrs(ld, "mean", "rdisp")
        self.meandispnorm.link_from(*parents)
        return self.meandispnorm

    def link_avatar(self, *parents):
        """Avatar: a double-buffered copy of the loader's minibatch so the
        loader can serve the next one while the forwards run (rule 6: the
        loader is then linked from start_point, not from the repeater)."""
        from veles_amd.avatar import Avatar
        self._require("loader")
        self.avatar = Avatar(self)
        attrs = [a for a in ("minibatch_data", "minibatch_labels",
                             "minibatch_targets", "minibatch_indices",
                             "minibatch_class", "minibatch_size",
                             "minibatch_offset", "last_minibatch",
                             "epoch_ended", "epoch_number", "class_lengths")
                 if getattr(self.loader, a, None) is not None]
        self.avatar.clone(self.loader, *attrs)
        self.avatar.link_from(*parents)
        return self.avatar

    def link_data_saver(self, *parents):
        """MinibatchesSaver of every served minibatch (rule 15)."""
        from veles_amd.loader.saver import MinibatchesSaver
        self._require("loader")
        cfg = dict(getattr(self, "data_saver_config", None) or {})
        self.data_saver = MinibatchesSaver(self, **cfg)
        self.data_saver.link_attrs(self.loader, "minibatch_data",
                                   "minibatch_size", "minibatch_class",
                                   "minibatch_indices")
        for a in ("minibatch_labels", "minibatch_targets"):
            if getattr(self.loader, a, None) is not None:
                self.data_saver.link_attrs(self.loader, a)
        self.data_saver.link_from(*parents)
        return self.data_saver

    link_datasaver = link_data_saver

    def link_image_saver(self, *parents):
        """ImageSaver of the misclassified inputs of an improving epoch
        (rule 10)."""
        from veles_amd.models.image_saver import ImageSaver
        self._require("loader", "decision")
        if not self.forwards:
            raise AttributeError("link the forwards first")
        cfg = dict(getattr(self, "image_saver_config", None) or {})
        self.image_saver = ImageSaver(self, **cfg)
        src = getattr(self, "meandispnorm", None)
        if src is not None:
            self.image_saver.link_attrs(src, ("input", "output"))
        else:
            self.image_saver.link_attrs(self.loader,
                                        ("input", "minibatch_data"))
        self.image_saver.link_attrs(self.forwards[-1], "output")
        self.image_saver.link_attrs(self.loader, "minibatch_class",
                                    "minibatch_size", "minibatch_offset",
                                    ("indices", "minibatch_indices"))
        if self.loss_function == "mse":
            self.image_saver.link_attrs(self.loader,
                                        ("target", "minibatch_targets"))
        else:
            self.image_saver.link_attrs(self.loader,
                                        ("labels", "minibatch_labels"))
        self.image_saver.gate_skip = ~self.decision.improved
        self.image_saver.link_from(*parents)
        return self.image_saver

    # -- services ---------------------------------------------------------
    def link_ipython(self, *parents):
        """Interactive shell (rule 13): opened on SIGUSR2 or with
        ``root.common.interactive``."""
        from veles_amd.interaction import Shell
        self._require("decision")
        self.ipython = Shell(self)
        self.ipython.link_from(*parents)
        return self.ipython

    def link_publisher(self, *parents):
        """Report of the run (config, results, timings, plots, graph),
        written once training completes."""
        from veles_amd.publishing import Publisher
        self._require("decision")
        cfg = dict(getattr(self, "publisher_config", None) or {})
        cfg.setdefault("plotters", [u for u in self if hasattr(u, "files") and
                                    hasattr(u, "redraw_threshold")])
        self.publisher = Publisher(self, **cfg)
        self.publisher.gate_block = ~self.decision.complete
        self.publisher.link_from(*parents)
        return self.publisher

    def link_result_unit(self, *parents, **kwargs):
        """ForwardWorkflowExtractor (rule 14): keeps (and optionally
        exports) the inference workflow of the trained layers."""
        from veles_amd.models.forward_workflow import \
            ForwardWorkflowExtractor
        self._require("decision")
        cfg = dict(getattr(self, "result_unit_config", None) or {})
        cfg.update(kwargs)
        cfg.setdefault("loader_name", self.loader_name)
        cfg.setdefault("loader_config", self.loader_config)
        self.result_unit = ForwardWorkflowExtractor(self, **cfg)
        self.result_unit.decision = self.decision
        self.result_unit.link_from(*parents)
        return self.result_unit

    # -- plotters (rules 16-20) -------------------------------------------
    def link_error_plotter(self, *parents):
        """Error percentage per epoch, one series per class that has
        samples (validation, train and test)."""
        from veles_amd.plotting_units import AccumulatingPlotter
        self._require("decision")
        self.error_plotters = []
        for cls in (VALID, TRAIN, TEST):
            p = AccumulatingPlotter(self, name="errors %s" % CLASS_NAME[cls],
                                    plot_name="%s error, %%" %
                                    CLASS_NAME[cls], input_field=cls)
            p.link_attrs(self.decision, ("input", "epoch_n_err_pt"))
            self.error_plotters.append(self._epoch_plotter_gate(p))
        return self._chain(self.error_plotters, parents)

    def link_conf_matrix_plotter(self, *parents):
        """The validation confusion matrix (the evaluator collects it:
        ``compute_confusion_matrix`` is switched on)."""
        from veles_amd.plotting_units import MatrixPlotter
        self._require("decision", "evaluator")
        self.evaluator.compute_confusion_matrix = True
        self.conf_matrix_plotter = MatrixPlotter(self, name="confusion matrix")
        self.conf_matrix_plotter.link_attrs(self.evaluator,
                                            ("input", "confusion_matrix"))
        self._epoch_plotter_gate(self.conf_matrix_plotter)
        self.conf_matrix_plotter.link_from(*parents)
        return self.conf_matrix_plotter

    def _mse_series(self, attr, title, parents, store):
        from veles_amd.plotting_units import AccumulatingPlotter
        self._require("decision")
        if not hasattr(self.decision, attr):
            raise AttributeError("%s needs an MSE decision (loss_function="
                                 "'mse')" % title)
        plots = []
        for cls in (VALID, TRAIN):
            p = AccumulatingPlotter(self, name="%s %s" % (title,
                                                          CLASS_NAME[cls]),
                                    input_field=cls)
            p.link_attrs(self.decision, ("input", attr))
            plots.append(self._epoch_plotter_gate(p))
        setattr(self, store, plots)
        return self._chain(plots, parents)

    def link_mse_plotter(self, *parents):
        """MSE per epoch (validation, train)."""
        return self._mse_series("epoch_mse", "mse", parents, "mse_plotters")

    def link_err_y_plotter(self, *parents):
        """RMSE per epoch (validation, train)."""
        return self._mse_series("epoch_rmse", "rmse", parents,
                                "err_y_plotters")

    def link_min_max_plotter(self, *parents):
        """Minimum and maximum of the network output at every epoch end."""
        from veles_amd.plotting_units import AccumulatingPlotter
        self._require("decision")
        self.min_max_plotters = []
        for stat in ("max", "min"):
            p = AccumulatingPlotter(self, name="output %s" % stat,
                                    input_field=stat)
            p.link_attrs(self.forwards[-1], ("input", "output"))
            self.min_max_plotters.append(self._epoch_plotter_gate(p))
        return self._chain(self.min_max_plotters, parents)

    def link_multi_hist_plotter(self, *parents):
        """Per-neuron weight histograms of every weighted layer."""
        from veles_amd.plotting_units import MultiHistogram
        self._require("decision")
        self.multi_hist_plotters = []
        for f in self._weighted_forwards():
            p = MultiHistogram(self, name="histogram %s" % f.name,
                               limit=16, n_bars=20)
            p.source_unit = f
            p.input = _WeightsRef(f)
            self.multi_hist_plotters.append(self._epoch_plotter_gate(p))
        if not self.multi_hist_plotters:
            raise ValueError("link_multi_hist_plotter: no weighted layers")
        return self._chain(self.multi_hist_plotters, parents)

    def link_weights_plotter(self, *parents, limit=64, layer=0):
        """The first layer's kernels / neurons as images (rule 17)."""
        from veles_amd.plotting_units import Weights2D
        self._require("decision", "loader")
        wf = self._weighted_forwards()
        if not wf:
            raise ValueError("link_weights_plotter: no weighted layers")
        self.weights_plotter = Weights2D(self, name="weights %s" %
                                         wf[layer].name, limit=limit,
                                         source_unit=wf[layer])
        self._epoch_plotter_gate(self.weights_plotter)
        self.weights_plotter.link_from(*parents)
        return self.weights_plotter

    def link_similar_weights_plotter(self, *parents, limit=64):
        """The weights plotter's layer with neurons ordered by similarity
        (rule 18: link_weights_plotter first)."""
        from veles_amd.plotting_units import Weights2D
        self._require("weights_plotter")
        src = self.weights_plotter.source_unit
        self.similar_weights_plotter = Weights2D(
            self, name="similar weights %s" % src.name, limit=limit,
            similar=True, source_unit=src)
        self._epoch_plotter_gate(self.similar_weights_plotter)
        self.similar_weights_plotter.link_from(*parents)
        return self.similar_weights_plotter

    def link_image_plotter(self, *parents, limit=16):
        """The network output as images (auto-encoders, rule 19)."""
        from veles_amd.plotting_units import ImagePlotter
        self._require("decision")
        out = self.forwards[-1]
        self.image_plotter = ImagePlotter(self, name="output images",
                                          limit=limit)
        self.image_plotter.link_attrs(out, ("input", "output"))
        self._epoch_plotter_gate(self.image_plotter)
        self.image_plotter.link_from(*parents)
        return self.image_plotter

    def link_immediate_plotter(self, *parents):
        """Input, output (and target) of the first sample as curves
        (rule 17)."""
        from veles_amd.plotting_units import ImmediatePlotter
        self._require("decision", "loader")
        inputs = [self.loader.minibatch_data, self.forwards[-1].output]
        if getattr(self.loader, "minibatch_targets", None) is not None:
            inputs.append(self.loader.minibatch_targets)
        self.immediate_plotter = ImmediatePlotter(
            self, name="immediate", inputs=[_First(a) for a in inputs])
        self._epoch_plotter_gate(self.immediate_plotter)
        self.immediate_plotter.link_from(*parents)
        return self.immediate_plotter

    def link_table_plotter(self, *parents):
        """Max / min / mean / std of every layer's weights, outputs and
        weight gradients (rule 20: the GD units must exist)."""
        from veles_amd.plotting_units import TableMaxMin
        self._require("decision")
        if not self.gds:
            raise AttributeError("link the gradient descent units first")
        values = {}
        weighted = self._weighted_forwards()
        for f in self.forwards:
            if f in weighted:
                values["%s weights" % f.name] = _WeightsRef(f)
                values["%s gradient" % f.name] = _WeightsRef(f, "grad")
            if getattr(f, "output", None) is not None:
                values["%s output" % f.name] = f.output
        self.table_plotter = TableMaxMin(self, name="max min", values=values)
        self._epoch_plotter_gate(self.table_plotter)
        self.table_plotter.link_from(*parents)
        return self.table_plotter


class _WeightsRef(object):
    """A picklable handle that reads a layer's live weights (or their
    gradient) from the flat parameter store at plot time."""

    def __init__(self, unit, what="master"):
        self.unit = unit
        self.what = what

    def detach(self):
        p = getattr(self.unit, "_pw_", None)
        t = getattr(p, self.what, None) if p is not None else None
        if t is None:
            t = self.unit.weights.devmem
        if t is None:
            import torch
            t = torch.from_numpy(self.unit.weights.mem)
        return t.detach()


class _First(object):
    """The first sample of an Array (or tensor) at plot time."""

    def __init__(self, arr):
        self.arr = arr

    def detach(self):
        import torch
        a = self.arr
        t = getattr(a, "devmem", None)
        if t is None and getattr(a, "mem", None) is not None:
            t = torch.from_numpy(a.mem)
        return t[0].detach()
