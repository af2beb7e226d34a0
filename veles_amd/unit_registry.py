"""Metaclass registries with constructor-kwarg misprint detection.

Reference: veles/unit_registry.py:51-176 (``UnitRegistry``: every Unit subclass
is registered; the class' ``kwargs.get("...")`` keys are extracted so that a
misspelt constructor kwarg is reported with its closest valid spelling by
Damerau-Levenshtein distance), veles/mapped_object_registry.py:36-54.
"""
from __future__ import annotations

import inspect
import re
import threading

__all__ = ["UnitRegistry", "MappedUnitRegistry", "MappedObjectsRegistry",
           "damerau_levenshtein"]

_KWARG_RE = re.compile(r"""kwargs\.(?:get|pop|setdefault)\(\s*["'](\w+)["']""")
_KWARG_IDX_RE = re.compile(r"""kwargs\[\s*["'](\w+)["']\s*\]""")


def damerau_levenshtein(a, b):
    """Optimal-string-alignment Damerau-Levenshtein distance."""
    la, lb = len(a), len(b)
    d = [[0] * (lb + 1) for _ in range(la + 1)]
    for i in range(la + 1):
        d[i][0] = i
    for j in range(lb + 1):
        d[0][j] = j
    for i in range(1, la + 1):
        for j in range(1, lb + 1):
            cost = 0 if a[i - 1] == b[j - 1] else 1
            d[i][j] = min(d[i - 1][j] + 1, d[i][j - 1] + 1,
                          d[i - 1][j - 1] + cost)
            if (i > 1 and j > 1 and a[i - 1] == b[j - 2] and
                    a[i - 2] == b[j - 1]):
                d[i][j] = min(d[i][j], d[i - 2][j - 2] + cost)
    return d[la][lb]


def _scan_kwargs(cls):
    keys = set()
    for klass in cls.__mro__:
        if klass is object:
            continue
        try:
            src = inspect.getsource(klass)
        except (OSError, TypeError):
            continue
        keys.update(_KWARG_RE.findall(src))
        keys.update(_KWARG_IDX_RE.findall(src))
    return keys


class UnitRegistry(type):
    """Registers every non-hidden class; checks constructor kwargs."""

    units = set()
    _lock = threading.Lock()
    _kwarg_cache = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        if not clsdict.get("hide_from_registry", False):
            with UnitRegistry._lock:
                UnitRegistry.units.add(cls)

    def __call__(cls, *args, **kwargs):
        if kwargs and not getattr(cls, "disable_misprint_check", False):
            cls.check_misprints(kwargs)
        return super().__call__(*args, **kwargs)

    def known_kwargs(cls):
        keys = UnitRegistry._kwarg_cache.get(cls)
        if keys is None:
            keys = _scan_kwargs(cls)
            keys.update(getattr(cls, "KNOWN_KWARGS", ()))
            UnitRegistry._kwarg_cache[cls] = keys
        return keys

    def check_misprints(cls, kwargs):
        known = cls.known_kwargs()
        if not known:
            return []
        found = []
        for k in kwargs:
            if k in known:
                continue
            best = min(known, key=lambda x: damerau_levenshtein(k, x))
            dist = damerau_levenshtein(k, best)
            if dist <= max(1, len(k) // 4):
                found.append((k, best))
                import logging
                logging.getLogger(cls.__name__).warning(
                    "Unknown kwarg '%s' - did you mean '%s'?", k, best)
        return found


class MappedUnitRegistry(UnitRegistry):
    """Unit registry that also maps ``MAPPING`` names to classes."""

    mapped = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        mapping = clsdict.get("MAPPING")
        if mapping:
            if isinstance(mapping, str):
                mapping = (mapping,)
            for m in mapping:
                MappedUnitRegistry.mapped[m] = cls


class MappedObjectsRegistry(type):
    """Generic ``name -> class`` registry keyed by ``MAPPING``; subclasses set
    ``registry_name`` to get their own mapping dict."""

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        if not hasattr(cls, "registry"):
            cls.registry = {}
        mapping = clsdict.get("MAPPING")
        if mapping:
            cls.registry[mapping] = cls
