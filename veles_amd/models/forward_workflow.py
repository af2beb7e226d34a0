"""Forward-only (inference) workflow built from a trained StandardWorkflow.

Reference: ``StandardWorkflow.extract_forward_workflow(loader_name,
loader_config, result_unit_factory, result_unit_config, cyclic)``
(docs/source/manualrst_veles_example_advanced.rst:327-377): a test-mode
workflow with a new loader, the trained layers, and a result unit.

The new forwards are fresh units of the same classes and kwargs whose
weights are seeded from the trained ones (host copies, then the usual flat
bf16 device store), so the trained workflow is left untouched.  The new
loader shares the trained loader's normalizer and label mapping
(``derive_from``).  ``cyclic=True`` keeps serving (interactive / RESTful
loaders block for the next request); otherwise one pass over the TEST set.
"""
from __future__ import annotations

from veles_amd.models.standard_workflow import StandardWorkflow
from veles_amd.units import Unit

__all__ = ["ForwardWorkflow", "ForwardWorkflowExtractor"]


class ForwardWorkflow(StandardWorkflow):
    def __init__(self, workflow, **kwargs):
        self.result_unit_factory = kwargs.pop("result_unit_factory", None)
        self.result_unit_config = dict(kwargs.pop("result_unit_config",
                                                  None) or {})
        self.cyclic = kwargs.pop("cyclic", False)
        kwargs["testing"] = True
        kwargs.setdefault("decision_config", {"max_epochs": None})
        super().__init__(workflow, **kwargs)

    def create_workflow(self):
        self.link_repeater(self.start_point)
        self.link_loader(self.repeater)
        last = self.link_forwards(("input", "minibatch_data"), self.loader)
        if self.result_unit_factory is not None:
            ru = self.result_unit_factory(self, **self.result_unit_config)
            ru.link_from(last)
            if hasattr(ru, "output") or "output" in getattr(
                    ru, "demanded", ()):
                ru.link_attrs(last, "output")
            self.result_unit = ru
            last = ru
        else:
            from veles_amd.models.result_collector import OutputCollector
            ru = OutputCollector(self)
            ru.link_from(last)
            ru.link_attrs(last, "output")
            ru.link_attrs(self.loader, "minibatch_class", "minibatch_size",
                          "minibatch_indices")
            ru.labels_source = self.loader
            self.result_unit = self.output_collector = ru
            last = ru
        from veles_amd.mutable import Bool
        self.repeater.link_from(last)
        self.end_point.link_from(last)
        if self.cyclic:
            # serve until stopped (interactive / RESTful feeding)
            self.repeater.gate_block = Bool(False)
            self.end_point.gate_block = Bool(True)
        else:
            self.repeater.gate_block = self.loader.epoch_ended
            self.end_point.gate_block = ~self.loader.epoch_ended

    @classmethod
    def from_trained(cls, trained, loader_name, loader_config,
                     result_unit_factory=None, result_unit_config=None,
                     cyclic=False):
        fwd = cls(trained.workflow, layers=trained.layers,
                  loader_name=loader_name, loader_config=dict(loader_config),
                  loss_function=trained.loss_function,
                  result_unit_factory=result_unit_factory,
                  result_unit_config=result_unit_config, cyclic=cyclic)
        for src, dst in zip(trained.forwards, fwd.forwards):
            if hasattr(src, "sync_params_to_host"):
                src.sync_params_to_host()
                if src.weights.mem is not None:
                    dst.weights.reset(src.weights.mem.copy())
                if getattr(src, "include_bias", False) and \
                        src.bias.mem is not None:
                    dst.bias.reset(src.bias.mem.copy())
        fwd.loader.derive_from(trained.loader)
        return fwd


class ForwardWorkflowExtractor(Unit):
    """``StandardWorkflow.link_result_unit`` (reference docs
    manualrst_veles_workflow_creation.rst:520-533): keeps an inference
    workflow extracted from the training one - once training completes, or
    at every epoch that improved the validation error
    (``on_improvement=True``) - and optionally exports it as a libVeles-style
    package (``package=path.zip|.tar.gz``, read by the native runtime).

    Linked after the decision; the unit decides from ``decision.complete`` /
    ``decision.improved`` itself, so it can sit on any branch of the cycle.
    """
    MAPPING = "forward_workflow_extractor"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.loader_name = kwargs.get("loader_name")
        self.loader_config = kwargs.get("loader_config")
        self.result_unit_factory = kwargs.get("result_unit_factory")
        self.result_unit_config = kwargs.get("result_unit_config")
        self.package = kwargs.get("package")
        self.precision = kwargs.get("precision", 32)
        self.on_improvement = kwargs.get("on_improvement", False)
        self.extractions = 0
        self.demand("decision")

    def init_unpickled(self):
        super().init_unpickled()
        self.forward_workflow_ = None

    @property
    def forward_workflow(self):
        return self.forward_workflow_

    def run(self):
        d = self.decision
        due = bool(d.improved) if self.on_improvement else bool(d.complete)
        if not due:
            return
        wf = self.workflow
        self.forward_workflow_ = wf.extract_forward_workflow(
            self.loader_name, self.loader_config, self.result_unit_factory,
            self.result_unit_config)
        self.extractions += 1
        if self.package:
            self.forward_workflow_.package_export(
                self.package, precision=self.precision,
                archive_format="zip" if self.package.endswith(".zip")
                else "tgz")
            self.info("Exported the forward workflow to %s", self.package)
