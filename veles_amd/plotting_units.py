"""Plotting units (reference veles/plotting_units.py:52-903): accumulating
line plots of metrics, matrices (confusion / weights), image grids
(weights / minibatches), histograms, max-min tables.  All render to files
through :class:`veles_amd.plotter.Plotter`."""
from __future__ import annotations

import numpy

from veles_amd.plotter import Plotter

__all__ = ["AccumulatingPlotter", "MatrixPlotter", "ImagePlotter",
           "ImmediatePlotter", "Histogram", "AutoHistogramPlotter",
           "MultiHistogram", "TableMaxMin", "to_numpy"]


def to_numpy(v):
    if v is None:
        return None
    t = getattr(v, "devmem", None)
    if t is not None:
        return t.detach().float().cpu().numpy()
    m = getattr(v, "mem", None)
    if m is not None:
        return numpy.asarray(m)
    if hasattr(v, "detach"):
        return v.detach().float().cpu().numpy()
    return numpy.asarray(v)


class AccumulatingPlotter(Plotter):
    """Appends ``input`` (a scalar, or ``input[input_field]``) every run and
    draws the series (e.g. validation error per epoch)."""
    MAPPING = "accumulating_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.plot_name = kwargs.get("plot_name", self.name)
        self.input_field = kwargs.get("input_field")
        self.ylim = kwargs.get("ylim")
        self.values = []
        self.demand("input")

    def run(self):
        v = self.input
        if self.input_field is not None:
            v = v[self.input_field]
        self.values.append(float(numpy.asarray(to_numpy(v)).reshape(-1)[0]))
        super().run()

    def draw(self, fig):
        ax = fig.add_subplot(111)
        ax.plot(range(len(self.values)), self.values, marker="o")
        ax.set_title(self.plot_name)
        ax.grid(True)
        if self.ylim:
            ax.set_ylim(*self.ylim)


class MatrixPlotter(Plotter):
    """A 2-D matrix with values (confusion matrix)."""
    MAPPING = "matrix_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("input")

    def collect(self):
        self.matrix_ = to_numpy(self.input)

    def draw(self, fig):
        m = numpy.asarray(self.matrix_)
        ax = fig.add_subplot(111)
        im = ax.imshow(m, cmap="viridis")
        fig.colorbar(im)
        if m.size <= 400:
            for (i, j), v in numpy.ndenumerate(m):
                ax.text(j, i, "%g" % v, ha="center", va="center",
                        fontsize=6, color="w")


class ImagePlotter(Plotter):
    """A grid of the first ``limit`` samples / kernels of ``input``
    (NHWC images or [N, features] rows reshaped by ``sample_shape``)."""
    MAPPING = "image_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.limit = kwargs.get("limit", 16)
        self.sample_shape = kwargs.get("sample_shape")
        self.demand("input")

    def collect(self):
        a = to_numpy(self.input)[:self.limit]
        if self.sample_shape is not None:
            a = a.reshape((len(a),) + tuple(self.sample_shape))
        self.images_ = a

    def draw(self, fig):
        a = self.images_
        n = len(a)
        cols = int(numpy.ceil(numpy.sqrt(n)))
        rows = int(numpy.ceil(n / max(cols, 1)))
        for i in range(n):
            ax = fig.add_subplot(rows, cols, i + 1)
            img = a[i]
            if img.ndim == 3 and img.shape[-1] not in (1, 3):
                img = img[..., 0]
            if img.ndim == 3 and img.shape[-1] == 1:
                img = img[..., 0]
            lo, hi = float(img.min()), float(img.max())
            ax.imshow((img - lo) / (hi - lo + 1e-12), cmap="gray")
            ax.axis("off")


class ImmediatePlotter(Plotter):
    """Draws the current ``inputs`` (several 1-D series) as lines."""
    MAPPING = "immediate_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.inputs = list(kwargs.get("inputs", []))

    def collect(self):
        self.series_ = [numpy.asarray(to_numpy(v)).reshape(-1)
                        for v in self.inputs]

    def draw(self, fig):
        ax = fig.add_subplot(111)
        for s in self.series_:
            ax.plot(s)


class Histogram(Plotter):
    MAPPING = "histogram_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.n_bars = kwargs.get("n_bars", 30)
        self.demand("input")

    def collect(self):
        self.data_ = numpy.asarray(to_numpy(self.input)).reshape(-1)

    def draw(self, fig):
        ax = fig.add_subplot(111)
        ax.hist(self.data_, bins=self.n_bars)


class AutoHistogramPlotter(Histogram):
    """Histogram with the bar count chosen from the data (Freedman–
    Diaconis)."""
    MAPPING = "auto_histogram_plotter"

    def collect(self):
        super().collect()
        d = self.data_
        if d.size > 1:
            q75, q25 = numpy.percentile(d, [75, 25])
            w = 2 * (q75 - q25) / max(d.size, 1) ** (1 / 3)
            if w > 0:
                self.n_bars = int(min(200, max(5, (d.max() - d.min()) / w)))


class MultiHistogram(Plotter):
    """One histogram per row of ``input`` (e.g. weights of each neuron),
    up to ``limit``."""
    MAPPING = "multi_histogram_plotter"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.limit = kwargs.get("limit", 16)
        self.n_bars = kwargs.get("n_bars", 20)
        self.demand("input")

    def collect(self):
        a = numpy.asarray(to_numpy(self.input))
        self.rows_ = a.reshape(a.shape[0], -1)[:self.limit]

    def draw(self, fig):
        n = len(self.rows_)
        cols = int(numpy.ceil(numpy.sqrt(n)))
        rows = int(numpy.ceil(n / max(cols, 1)))
        for i, r in enumerate(self.rows_):
            ax = fig.add_subplot(rows, cols, i + 1)
            ax.hist(r, bins=self.n_bars)
            ax.set_xticks([])
            ax.set_yticks([])


class TableMaxMin(Plotter):
    """Max / min / mean / std of the linked arrays as a text table."""
    MAPPING = "table_max_min"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("format", "txt")
        super().__init__(workflow, **kwargs)
        self.values = dict(kwargs.get("values", {}))

    def collect(self):
        self.table_ = []
        for name, v in self.values.items():
            a = numpy.asarray(to_numpy(v), dtype=numpy.float64)
            self.table_.append((name, a.max(), a.min(), a.mean(), a.std()))

    def render(self):
        import os
        os.makedirs(self.directory, exist_ok=True)
        fn = os.path.join(self.directory, "%s%s.txt" % (self.name_prefix,
                                                       self.name))
        with open(fn, "w") as f:
            f.write("%-24s %12s %12s %12s %12s\n" % ("name", "max", "min",
                                                      "mean", "std"))
            for row in self.table_:
                f.write("%-24s %12.6g %12.6g %12.6g %12.6g\n" % row)
        if fn not in self.files:
            self.files.append(fn)
