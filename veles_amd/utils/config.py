"""Hierarchical auto-vivifying configuration tree (``root``).

Behavioural parity with the reference's config service
(reference: veles/config.py:60-176 for ``Config``/``get``/``validate_kwargs``,
veles/config.py:178-291 for the defaults, :293-308 site overrides, :319-321 protect).

Design differences (MI355X-first):
* ``root.common.engine`` describes the single HIP device layer (``backend`` in
  {"auto", "hip", "cpu"}), the compute ``precision_type`` (bfloat16 by default on the
  GPU, float32 on the CPU), the data-parallel knobs (``engine.dp.bucket_mb`` /
  ``overlap``) and the kernel-library knobs.  There is no OpenCL/CUDA/numba section.
* Nodes are plain Python objects; leaves are any value.  Reading a missing child
  creates an empty node (auto-vivification); ``get(node, default)`` turns an empty
  node into the default.
"""
from __future__ import annotations

import os
import pprint
import sys
import threading

__all__ = ["Config", "root", "get", "validate_kwargs", "fix_contents"]

_protected = {}
_lock = threading.RLock()


class Config(object):
    """A node of the configuration tree."""

    def __init__(self, path):
        object.__setattr__(self, "__path__", path)

    # -- mutation ---------------------------------------------------------
    def update(self, value):
        if self is root:
            raise ValueError("Root updates are disabled")
        if isinstance(value, Config):
            value = value.__content__
        if not isinstance(value, dict):
            raise ValueError("Value must be an instance of dict or Config")
        self.__update__(value)
        return self

    def __update__(self, tree):
        for k, v in tree.items():
            if isinstance(v, dict) and not v.get("dict", False):
                getattr(self, k).__update__(v)
            else:
                if isinstance(v, dict) and "dict" in v:
                    v = dict(v)
                    del v["dict"]
                setattr(self, k, v)

    def protect(self, *names):
        """Make the given child names read-only."""
        with _lock:
            _protected.setdefault(id(self), set()).update(names)

    # -- access -------------------------------------------------------------
    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)
        if name in ("keys", "values", "items"):
            return getattr(self.__content__, name)
        child = Config("%s.%s" % (self.__path__, name))
        object.__setattr__(self, name, child)
        return child

    def __setattr__(self, name, value):
        prot = _protected.get(id(self))
        if prot and name in prot:
            raise AttributeError(
                "Attempted to change the protected configuration setting "
                "%s.%s" % (self.__path__, name))
        object.__setattr__(self, name, value)

    def __getitem__(self, item):
        return getattr(self, item)

    def __setitem__(self, item, value):
        setattr(self, item, value)

    def __contains__(self, item):
        return item in self.__dict__ and item != "__path__"

    def __iter__(self):
        return iter(self.__content__)

    def __len__(self):
        return len(self.__content__)

    def __bool__(self):
        # An empty (auto-vivified) node is "undefined" and therefore falsy.
        return len(self.__content__) > 0

    @property
    def __content__(self):
        d = dict(self.__dict__)
        d.pop("__path__", None)
        return d

    def to_dict(self):
        return fix_contents(self)

    def print_(self, indent=1, width=80, file=sys.stdout):
        print("-" * width, file=file)
        print('Configuration "%s":' % self.__path__, file=file)
        pprint.pprint(fix_contents(self), indent=indent, width=width,
                      stream=file)
        print("-" * width, file=file)

    def __repr__(self):
        return '<Config "%s": %r>' % (self.__path__, self.__content__)

    # -- pickling -----------------------------------------------------------
    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, state):
        self.__dict__.update(state)


def fix_contents(cfg):
    """Convert a Config subtree into nested dicts (for printing / JSON)."""
    if not isinstance(cfg, Config):
        return cfg
    return {k: fix_contents(v) for k, v in cfg.__content__.items()}


def get(value, default_value=None):
    """Return ``default_value`` if ``value`` is an (undefined) Config node."""
    if isinstance(value, Config):
        return default_value
    return value


def validate_kwargs(caller, **kwargs):
    """Warn about kwargs bound to undefined config nodes (reference:
    veles/config.py:165-176)."""
    for k, v in kwargs.items():
        if isinstance(v, Config) and len(v.__content__) == 0:
            warn = getattr(caller, "warning", None)
            if warn is not None:
                warn("Argument '%s' seems to be undefined at %s", k,
                     v.__path__)


root = Config("root")

_home = os.path.join(os.path.expanduser("~"), ".veles_amd")
_pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

root.common.update({
    "dirs": {
        "veles": _pkg_root,
        "user": _home,
        "datasets": os.path.join(_home, "data"),
        "snapshots": os.path.join(_home, "snapshots"),
        "cache": os.path.join(_home, "cache"),
        "dist_config": "/etc/default/veles_amd",
    },
    "disable": {
        "spinning_run_progress": True,
        "plotting": True,
        "snapshotting": False,
        "publishing": False,
    },
    "trace": {
        "misprints": False,
        "undefined_configs": False,
        "run": False,
        # Chrome-trace JSON path for timeline events (None = off).
        "events_file": None,
    },
    "exceptions": {"run_after_stop": False},
    "timings": None,
    "api": {"port": 8180, "path": "/api"},
    "engine": {
        # "auto" picks "hip" when an MI355X is visible, otherwise "cpu".
        "backend": "auto",
        # Compute dtype of the matrix ops on the GPU.  The CPU reference path
        # always computes in float32.
        "precision_type": "bfloat16",
        # 0: fp32 MFMA accumulate; 1: split-K with compensated fp32 reduce
        # (reference precision levels, veles/config.py:247-251).
        "precision_level": 0,
        "device_id": None,
        "sync_run": False,
        # Capture the forward and backward unit chains of the train step in
        # HIP graphs on the GPU (veles_amd/graphs.py); VELES_AMD_GRAPHS=0
        # overrides.
        "graphs": True,
        "force_cpu": (),
        "thread_pool": {"minthreads": 2, "maxthreads": 2},
        "kernels": {
            # Where the compiled HIP kernel library lives (in-tree by default).
            "library": None,
            # Per-shape kernel selection table (tile configs); see
            # veles_amd/ops/autotune.py.
            "tuning_file": None,
        },
        "dp": {
            # Gradient all-reduce bucket size (MB of fp32).  xGMI is point-to-
            # point: 32-64 MB buckets keep every link busy; see
            # docs/PARALLEL.md for the derivation.
            "bucket_mb": 32,
            # MB of the last bucket (the layers whose gradients come last):
            # the only all-reduce that cannot overlap the backward pass
            "tail_bucket_mb": 2,
            # multi-rank: update each bucket on a side stream as soon as its
            # all-reduce is done (ParameterStore._bucket_update); False keeps
            # one fused update after the last all-reduce
            "overlap": True,
            "timeout_s": 600,
        },
    },
    "genetics": {"disable": {"plotting": True}},
    "ensemble": {"disable": {"plotting": True}},
})


def _apply_site_configs():
    import runpy
    for d in (root.common.dirs.dist_config, _home, os.getcwd()):
        path = os.path.join(d, "site_config.py")
        if os.path.isfile(path):
            try:
                ns = runpy.run_path(path)
                if "update" in ns:
                    ns["update"](root)
            except Exception as e:  # pragma: no cover - user file
                print("Failed to apply %s: %s" % (path, e), file=sys.stderr)


if os.environ.get("VELES_AMD_NO_SITE_CONFIG") is None:
    _apply_site_configs()
