"""Plotting units (reference veles/plotting_units.py:52-903): accumulating
line plots of metrics, matrices (confusion / weights), image grids
(weights / minibatches), histograms, max-min tables.  All render to files
through :class:`veles_amd.plotter.Plotter`."""
from __future__ import annotations

import numpy

from veles_amd.plotter import Plotter

__all__ = ["AccumulatingPlotter", "MatrixPlotter", "ImagePlotter",
           "ImmediatePlotter", "Histogram", "AutoHistogramPlotter",
           "MultiHistogram", "TableMaxMin", "Weights2D", "to_numpy",
           "unit_weights"]

# scalar reductions an AccumulatingPlotter can apply to an array input
_REDUCE = {"max": numpy.max, "min": numpy.min, "mean": numpy.mean,
           "norm": lambda a: float(numpy.sqrt(numpy.sum(a * a)))}


def unit_weights(unit, name="weights"):
    """The live weights of a forward unit: the device master copy of the
    flat parameter store when it exists (``Array.mem`` is only synced for
    snapshots), else the unit's Array."""
    p = getattr(unit, {"weights": "_pw_", "bias": "_pb_"}.get(name, ""),
                None)
    if p is not None and p.master is not None:
        return p.master
    return getattr(unit, name)


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
        if self.input_field in _REDUCE:
            # a statistic of an array (min / max of an output, weight norm)
            a = numpy.asarray(to_numpy(v), dtype=numpy.float64).reshape(-1)
            self.values.append(float(_REDUCE[self.input_field](a)))
        else:
            if self.input_field is not None:
                v = v[self.input_field]
            self.values.append(float(numpy.asarray(
                to_numpy(v)).reshape(-1)[0]))
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
        elif a.ndim == 2:
            # flat samples (FC outputs): zero-padded square images
            side = int(numpy.ceil(numpy.sqrt(a.shape[1])))
            sq = numpy.zeros((len(a), side * side), a.dtype)
            sq[:, :a.shape[1]] = a
            a = sq.reshape(len(a), side, side)
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
        fn = os.path.join(self.directory, "%s%s.txt" % (
            self.name_prefix, self.name.replace(" ", "_")))
        with open(fn, "w") as f:
            f.write("%-24s %12s %12s %12s %12s\n" % ("name", "max", "min",
                                                      "mean", "std"))
            for row in self.table_:
                f.write("%-24s %12.6g %12.6g %12.6g %12.6g\n" % row)
        if fn not in self.files:
            self.files.append(fn)


class Weights2D(Plotter):
    """The first ``limit`` kernels / neurons of a layer's weights as images
    (Znicz ``Weights2D``, ``link_weights_plotter``): conv kernels
    [OC][KH][KW][C] are drawn as KHxKW(xC) images, fully-connected rows as
    ``sample_shape`` images (the layer's input sample shape by default).

    ``similar=True`` orders the neurons so that the most similar pairs
    (cosine similarity of their weight rows) are adjacent - the
    ``link_similar_weights_plotter`` view used to spot duplicated units.
    The source is a forward unit; its live device weights are read at draw
    time (``unit_weights``)."""
    MAPPING = "weights_2d"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.limit = kwargs.get("limit", 64)
        self.sample_shape = kwargs.get("sample_shape")
        self.similar = kwargs.get("similar", False)
        self.weights_name = kwargs.get("weights_name", "weights")
        self.source_unit = kwargs.get("source_unit")

    def collect(self):
        w = numpy.asarray(to_numpy(unit_weights(self.source_unit,
                                                self.weights_name)))
        rows = w.reshape(w.shape[0], -1)
        if self.similar and len(rows) > 1:
            rows = rows[similarity_order(rows)]
        rows = rows[:self.limit]
        if w.ndim == 4:
            imgs = rows.reshape((len(rows),) + w.shape[1:])
        else:
            shape = self.sample_shape
            if shape is None:
                inp = getattr(self.source_unit, "input", None)
                shp = getattr(inp, "shape", None)
                shape = tuple(shp[1:]) if shp is not None and \
                    int(numpy.prod(shp[1:])) == rows.shape[1] else None
            if shape is None:
                side = int(numpy.ceil(numpy.sqrt(rows.shape[1])))
                pad = numpy.zeros((len(rows), side * side), rows.dtype)
                pad[:, :rows.shape[1]] = rows
                rows, shape = pad, (side, side)
            imgs = rows.reshape((len(rows),) + tuple(shape))
        self.images_ = imgs

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


def similarity_order(rows):
    """A greedy chain through the rows: start from the most similar pair
    (cosine), then always append the row most similar to the chain's end."""
    r = numpy.asarray(rows, dtype=numpy.float64)
    nrm = numpy.linalg.norm(r, axis=1, keepdims=True)
    u = r / numpy.where(nrm > 0, nrm, 1.0)
    sim = u @ u.T
    numpy.fill_diagonal(sim, -numpy.inf)
    i, j = numpy.unravel_index(int(numpy.argmax(sim)), sim.shape)
    order = [int(i), int(j)]
    used = numpy.zeros(len(r), bool)
    used[order] = True
    while len(order) < len(r):
        cand = numpy.where(used, -numpy.inf, sim[order[-1]])
        k = int(numpy.argmax(cand))
        order.append(k)
        used[k] = True
    return numpy.asarray(order)
