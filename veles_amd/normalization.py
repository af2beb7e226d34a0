"""Dataset normalizers (registry by name).

Reference: veles/normalization.py:57-662.  Registry names and formulas kept:
``mean_disp`` ((x - mean) / (max - min), per feature), ``linear`` (per-sample
map of [min, max] onto an interval), ``range_linear`` (dataset-wide
[min, max] onto an interval), ``exp`` (per-sample softmax-like), ``none``,
``pointwise`` (per-feature affine onto [-1, 1]), ``external_mean`` (subtract a
given mean image, optional scale), ``internal_mean`` (subtract the dataset mean).

Normalizers whose effect is a per-feature affine map expose
``affine() -> (mean, rdisp)`` so the GPU minibatch gather can apply them on
the fly to uint8 data kept resident in HBM (``out = (x - mean) * rdisp``).
"""
from __future__ import annotations

import numpy

__all__ = ["NormalizerRegistry", "NormalizerBase", "normalizer",
           "UninitializedStateError"]


class UninitializedStateError(Exception):
    pass


class NormalizerRegistry(type):
    normalizers = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        m = clsdict.get("MAPPING")
        if m:
            NormalizerRegistry.normalizers[m] = cls


def normalizer(name, **kwargs):
    try:
        return NormalizerRegistry.normalizers[name](**kwargs)
    except KeyError:
        raise ValueError("Unknown normalization type %r (known: %s)" %
                         (name, sorted(NormalizerRegistry.normalizers)))


def _prep(data):
    """Collapse all but the first axis: [N, features]."""
    return data.reshape(data.shape[0], -1)


class NormalizerBase(object, metaclass=NormalizerRegistry):
    MAPPING = None
    stateless = False

    def __init__(self, **kwargs):
        self._initialized = False
        self.reset()

    def reset(self):
        self._initialized = False

    @property
    def is_initialized(self):
        return self._initialized

    def analyze(self, data):
        self._initialized = True

    def normalize(self, data):
        if not self._initialized and not self.stateless:
            raise UninitializedStateError(
                "%s: analyze() was never called" % type(self).__name__)
        return self._normalize(data)

    def analyze_and_normalize(self, data):
        self.analyze(data)
        return self.normalize(data)

    def denormalize(self, data, **kwargs):
        return self._denormalize(data, **kwargs)

    def _normalize(self, data):
        return data

    def _denormalize(self, data, **kwargs):
        return data

    def affine(self):
        """(mean, rdisp) float32 per-feature arrays or None."""
        return None

    @property
    def state(self):
        return {k: v for k, v in self.__dict__.items()}

    @state.setter
    def state(self, value):
        self.__dict__.update(value)
        self._initialized = True


class StatelessNormalizer(NormalizerBase):
    stateless = True

    def analyze(self, data):
        self._initialized = True


class NoneNormalizer(StatelessNormalizer):
    MAPPING = "none"


class MeanDispersionNormalizer(NormalizerBase):
    """(x - mean) / (max - min) per feature (reference normalization.py:284)."""
    MAPPING = "mean_disp"

    def reset(self):
        super().reset()
        self._sum = None
        self._count = 0
        self._min = None
        self._max = None

    def analyze(self, data):
        d = _prep(data).astype(numpy.float64)
        if self._sum is None:
            self._sum = d.sum(0)
            self._min = d.min(0)
            self._max = d.max(0)
        else:
            self._sum += d.sum(0)
            self._min = numpy.minimum(self._min, d.min(0))
            self._max = numpy.maximum(self._max, d.max(0))
        self._count += d.shape[0]
        self._initialized = True

    def coefficients(self):
        mean = self._sum / max(self._count, 1)
        disp = self._max - self._min
        return mean, disp

    def affine(self):
        mean, disp = self.coefficients()
        rdisp = numpy.where(disp > 0, 1.0 / numpy.where(disp > 0, disp, 1),
                            1.0)
        return mean.astype(numpy.float32), rdisp.astype(numpy.float32)

    def _normalize(self, data):
        mean, rdisp = self.affine()
        d = _prep(data)
        d -= mean.astype(d.dtype)
        d *= rdisp.astype(d.dtype)
        return data

    def _denormalize(self, data, **kwargs):
        mean, rdisp = self.affine()
        d = _prep(data)
        d /= rdisp.astype(d.dtype)
        d += mean.astype(d.dtype)
        return data


class IntervalMixin(object):
    def _set_interval(self, kwargs):
        self.interval = tuple(kwargs.get("interval", (-1, 1)))


class LinearNormalizer(StatelessNormalizer, IntervalMixin):
    """Per-sample linear map of [min, max] onto ``interval``."""
    MAPPING = "linear"

    def __init__(self, **kwargs):
        self._set_interval(kwargs)
        super().__init__(**kwargs)

    def _normalize(self, data):
        d = _prep(data)
        imin, imax = self.interval
        dmin = d.min(1, keepdims=True)
        dmax = d.max(1, keepdims=True)
        diff = numpy.where(dmax > dmin, dmax - dmin, 1)
        d *= (imax - imin) / diff
        d += imin - dmin * (imax - imin) / diff
        return data


class RangeLinearNormalizer(NormalizerBase, IntervalMixin):
    """Dataset-wide [min, max] onto ``interval``."""
    MAPPING = "range_linear"

    def __init__(self, **kwargs):
        self._set_interval(kwargs)
        super().__init__(**kwargs)

    def reset(self):
        super().reset()
        self.min = None
        self.max = None

    def analyze(self, data):
        mn, mx = float(numpy.min(data)), float(numpy.max(data))
        self.min = mn if self.min is None else min(self.min, mn)
        self.max = mx if self.max is None else max(self.max, mx)
        self._initialized = True

    def _coef(self):
        imin, imax = self.interval
        diff = (self.max - self.min) or 1.0
        mul = (imax - imin) / diff
        return mul, imin - self.min * mul

    def affine(self):
        mul, add = self._coef()
        # (x - mean) * rdisp == x*mul + add  ->  mean = -add/mul, rdisp = mul
        return (numpy.float32(-add / mul) if mul else numpy.float32(0),
                numpy.float32(mul))

    def _normalize(self, data):
        mul, add = self._coef()
        data *= mul
        data += add
        return data

    def _denormalize(self, data, **kwargs):
        mul, add = self._coef()
        data -= add
        data /= mul
        return data


class ExponentNormalizer(StatelessNormalizer):
    MAPPING = "exp"

    def _normalize(self, data):
        d = _prep(data)
        d -= d.max(1, keepdims=True)
        numpy.exp(d, d)
        d /= d.sum(1, keepdims=True)
        return data


class PointwiseNormalizer(NormalizerBase):
    """Per-feature affine onto [-1, 1] from the observed min/max."""
    MAPPING = "pointwise"

    def reset(self):
        super().reset()
        self._min = None
        self._max = None

    def analyze(self, data):
        d = _prep(data)
        mn, mx = d.min(0), d.max(0)
        self._min = mn if self._min is None else numpy.minimum(self._min, mn)
        self._max = mx if self._max is None else numpy.maximum(self._max, mx)
        self._initialized = True

    def _coef(self):
        diff = (self._max - self._min).astype(numpy.float64)
        mul = numpy.where(diff > 0, 2.0 / numpy.where(diff > 0, diff, 1), 1.0)
        add = -1.0 - self._min * mul
        add = numpy.where(diff > 0, add, 0.0)
        return mul, add

    def affine(self):
        mul, add = self._coef()
        return (-add / mul).astype(numpy.float32), mul.astype(numpy.float32)

    def _normalize(self, data):
        mul, add = self._coef()
        d = _prep(data)
        d *= mul.astype(d.dtype)
        d += add.astype(d.dtype)
        return data

    def _denormalize(self, data, **kwargs):
        mul, add = self._coef()
        d = _prep(data)
        d -= add.astype(d.dtype)
        d /= mul.astype(d.dtype)
        return data


class ExternalMeanNormalizer(StatelessNormalizer):
    """Subtract a given mean sample (e.g. an ImageNet mean image), then
    multiply by ``scale``."""
    MAPPING = "external_mean"

    def __init__(self, **kwargs):
        mean = kwargs.get("mean_source")
        if isinstance(mean, str):
            mean = numpy.load(mean, allow_pickle=False)
        self.mean = None if mean is None else numpy.asarray(mean, numpy.float32)
        self.scale = float(kwargs.get("scale", 1.0))
        super().__init__(**kwargs)

    def affine(self):
        if self.mean is None:
            return None
        return (self.mean.ravel(),
                numpy.full(self.mean.size, self.scale, numpy.float32))

    def _normalize(self, data):
        d = _prep(data)
        d -= self.mean.ravel().astype(d.dtype)
        d *= self.scale
        return data

    def _denormalize(self, data, **kwargs):
        d = _prep(data)
        d /= self.scale
        d += self.mean.ravel().astype(d.dtype)
        return data


class InternalMeanNormalizer(NormalizerBase):
    MAPPING = "internal_mean"

    def __init__(self, **kwargs):
        self.scale = float(kwargs.get("scale", 1.0))
        super().__init__(**kwargs)

    def reset(self):
        super().reset()
        self._sum = None
        self._count = 0

    def analyze(self, data):
        d = _prep(data).astype(numpy.float64)
        self._sum = d.sum(0) if self._sum is None else self._sum + d.sum(0)
        self._count += d.shape[0]
        self._initialized = True

    def affine(self):
        mean = (self._sum / max(self._count, 1)).astype(numpy.float32)
        return mean, numpy.full(mean.size, self.scale, numpy.float32)

    def _normalize(self, data):
        mean, sc = self.affine()
        d = _prep(data)
        d -= mean.astype(d.dtype)
        d *= self.scale
        return data

    def _denormalize(self, data, **kwargs):
        mean, sc = self.affine()
        d = _prep(data)
        d /= self.scale
        d += mean.astype(d.dtype)
        return data
