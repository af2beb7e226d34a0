"""Tuneable config leaves for the genetic optimizer (reference
veles/genetics/config.py:45-227: ``Range``/``Tuneable``, ``fix_config``
replaces them by their defaults for normal runs, __main__.py:719-721)."""
from __future__ import annotations

from veles_amd.utils.config import Config

__all__ = ["Tuneable", "Range", "fix_config", "find_tuneables",
           "set_tuneables"]


class Tuneable(object):
    def __init__(self, default):
        self.default = default

    def __repr__(self):
        return "%s(%r)" % (type(self).__name__, self.default)


class Range(Tuneable):
    """A numeric hyper-parameter in [min_value, max_value]."""

    def __init__(self, default, min_value=None, max_value=None):
        super().__init__(default)
        if min_value is None:
            min_value = default / 10 if default else 0.0
        if max_value is None:
            max_value = default * 10 if default else 1.0
        if not min_value <= default <= max_value:
            raise ValueError("default outside [min, max]")
        self.min_value = min_value
        self.max_value = max_value
        self.is_int = isinstance(default, int) and isinstance(
            min_value, int) and isinstance(max_value, int)


def _walk(node, path=()):
    if isinstance(node, Config):
        for k, v in node.__content__.items():
            yield from _walk(v, path + (k,))
    elif isinstance(node, dict):
        for k, v in node.items():
            yield from _walk(v, path + (k,))
    elif isinstance(node, (list, tuple)):
        for i, v in enumerate(node):
            yield from _walk(v, path + (i,))
    else:
        yield path, node


def find_tuneables(cfg):
    return [(p, v) for p, v in _walk(cfg) if isinstance(v, Tuneable)]


def _set(cfg, path, value):
    node = cfg
    for k in path[:-1]:
        node = node[k] if not isinstance(node, Config) else getattr(node, k)
    last = path[-1]
    if isinstance(node, Config):
        setattr(node, last, value)
    else:
        node[last] = value


def set_tuneables(cfg, values):
    for (path, _), v in zip(find_tuneables(cfg), values):
        _set(cfg, path, v)


def fix_config(cfg):
    """Replace every Tuneable by its default (normal, non-GA runs)."""
    for path, t in find_tuneables(cfg):
        _set(cfg, path, t.default)
