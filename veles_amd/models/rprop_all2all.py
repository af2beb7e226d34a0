"""RPropAll2All: the backward of a fully connected layer trained with
resilient propagation (Znicz ``rprop_all2all``,
docs/source/manualrst_veles_workflow_parameters.rst:482).

Gradients are produced exactly like ``GradientDescent`` (one MFMA GEMM with
the bias gradient fused in); the update runs in the store's fused solver
kernel in iRprop- mode (ops.SOLVERS["rprop"]): per-weight step sizes grow
by 1.2 while the gradient sign holds and halve when it flips.  With data
parallelism the all-reduced gradient drives the step, so every rank keeps
identical steps.
"""
from __future__ import annotations

from veles_amd.models.gd import GradientDescent

__all__ = ["RPropAll2All"]


class RPropAll2All(GradientDescent):
    MAPPING = "rprop_all2all"
    SOLVER = "rprop"

    def __init__(self, workflow, **kwargs):
        # initial per-weight step (the solver's lr)
        kwargs.setdefault("learning_rate", 0.01)
        super().__init__(workflow, **kwargs)
