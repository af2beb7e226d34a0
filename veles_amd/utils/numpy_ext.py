"""numpy helpers (reference veles/numpy_ext.py:41-132)."""
from __future__ import annotations

import numpy

__all__ = ["roundup", "max_type", "eq_addr", "assert_addr", "ravel",
           "reshape", "transpose", "interleave", "NumDiff"]


def roundup(num, align):
    d = num % align
    return num if d == 0 else num + (align - d)


def max_type(num):
    """Largest absolute value a numpy dtype can hold."""
    if num.dtype.kind in "iu":
        return numpy.iinfo(num.dtype).max
    return numpy.finfo(num.dtype).max


def eq_addr(a, b):
    return a.__array_interface__["data"][0] == \
        b.__array_interface__["data"][0]


def assert_addr(a, b):
    if not eq_addr(a, b):
        raise ValueError("different buffers")


def ravel(a):
    b = a.ravel()
    assert_addr(a, b)
    return b


def reshape(a, shape):
    b = a.reshape(shape)
    assert_addr(a, b)
    return b


def transpose(a):
    b = a.transpose()
    assert_addr(a, b)
    return b


def interleave(arr):
    """[N, C, H, W] -> [N, H, W, C] (channel-last), a copy."""
    return numpy.ascontiguousarray(numpy.moveaxis(arr, 1, -1))


class NumDiff(object):
    """Numeric derivative by the 5-point stencil (used by gradient
    checks)."""
    h = 1.0e-3
    points = (2.0 * h, h, -h, -2.0 * h)
    coeffs = numpy.array([-1.0, 8.0, -8.0, 1.0]) / (12.0 * h)

    def __init__(self):
        self.errs = numpy.zeros(len(self.points))

    @property
    def derivative(self):
        return float((self.errs * self.coeffs).sum())

    def check_diff(self, x, y, target, f):
        """d f(x)/dx at ``x`` for a scalar loss f."""
        del y, target
        for i, p in enumerate(self.points):
            self.errs[i] = f(x + p)
        return self.derivative
