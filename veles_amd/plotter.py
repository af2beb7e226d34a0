"""Plotter base (reference veles/plotter.py:47-179).

The reference pickles each plotter to a ZeroMQ graphics server that renders
it with matplotlib in another process.  Here plotters render directly to
image files with matplotlib's Agg backend (headless GPU boxes), rate-limited
by ``redraw_threshold`` seconds, on rank 0 only, and only host copies of
small tensors are touched (metrics, a few weight rows), never the hot path.
``root.common.disable.plotting`` turns every plotter into a no-op.
"""
from __future__ import annotations

import os
import time

from veles_amd.units import Unit
from veles_amd.utils.config import get, root

__all__ = ["Plotter"]


class Plotter(Unit):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "PLOTTER")
        super().__init__(workflow, **kwargs)
        self.redraw_threshold = kwargs.get("redraw_threshold", 2.0)
        self.directory = kwargs.get("directory", get(
            root.common.dirs.plots, os.path.join(get(
                root.common.dirs.cache, "."), "plots")))
        self.file_format = kwargs.get("format", "png")
        self.name_prefix = kwargs.get("prefix", "")
        self.last_redraw = 0.0
        self.files = []

    def init_unpickled(self):
        super().init_unpickled()
        self.figure_ = None

    @property
    def disabled(self):
        if get(root.common.disable.plotting, False):
            return True
        launcher = getattr(self.workflow, "workflow", None)
        return getattr(launcher, "rank", 0) not in (0, None)

    def run(self):
        if self.disabled:
            return
        now = time.time()
        if now - self.last_redraw < self.redraw_threshold:
            return
        self.last_redraw = now
        self.collect()
        self.render()

    def collect(self):
        """Copy what will be drawn (host side)."""

    def draw(self, fig):
        raise NotImplementedError

    def render(self):
        import matplotlib
        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt
        fig = plt.figure(figsize=(6, 4))
        try:
            self.draw(fig)
            os.makedirs(self.directory, exist_ok=True)
            fn = os.path.join(self.directory, "%s%s.%s" % (
                self.name_prefix, self.name.replace(" ", "_"),
                self.file_format))
            fig.savefig(fn)
            if fn not in self.files:
                self.files.append(fn)
        finally:
            plt.close(fig)

    def stop(self):
        if not self.disabled and self.last_redraw:
            self.collect()
            self.render()
