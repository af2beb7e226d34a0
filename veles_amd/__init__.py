"""veles_amd - an MI355X-native dataflow deep-learning engine with the
Unit/Workflow programming model of Veles (devbib/veles).

See README.md for the architecture and SURVEY.md for the reference analysis.

The module itself is callable like the reference's (veles/__init__.py:
142-189): ``veles_amd("wf.py", "wf_config.py", "root.x=1", backend="cpu")``
runs the workflow in-process with the CLI semantics and returns the
``Main`` object (``.workflow``, ``.launcher``).
"""
import sys as _sys
import types as _types

__version__ = "0.1.0"
__all__ = ["__version__", "root"]

from veles_amd.utils.config import root  # noqa: E402,F401


class _VelesModule(_types.ModuleType):
    def __call__(self, workflow, config="-", *overrides, **kwargs):
        from veles_amd.__main__ import Main
        from veles_amd.cmdline import kwargs_to_argv
        argv = kwargs_to_argv(**kwargs) + [workflow, config] + \
            list(overrides)
        m = Main(argv)
        rc = m.run()
        if rc:
            raise RuntimeError("veles_amd(%s) exited with %s" % (workflow,
                                                                 rc))
        return m

    @property
    def __units__(self):
        """Every registered unit class (reference ``veles.__units__``)."""
        import importlib
        for m in ("veles_amd.models", "veles_amd.loader", "veles_amd.avatar",
                  "veles_amd.downloader", "veles_amd.input_joiner",
                  "veles_amd.mean_disp_normalizer", "veles_amd.plotting_units",
                  "veles_amd.snapshotter"):
            importlib.import_module(m)
        from veles_amd.unit_registry import UnitRegistry
        return set(UnitRegistry.units)


    @property
    def __loc__(self):
        """Non-blank, non-comment lines of the package per language
        (reference ``veles.__loc__``, veles/__init__.py:242-291)."""
        import os
        here = os.path.dirname(os.path.abspath(__file__))
        top = os.path.dirname(here)
        exts = {".py": "python", ".hip": "hip", ".h": "c++", ".cc": "c++"}
        out = {}
        for base in (here, os.path.join(top, "csrc")):
            for d, _, files in os.walk(base):
                for f in files:
                    lang = exts.get(os.path.splitext(f)[1])
                    if lang is None:
                        continue
                    cmt = "#" if lang == "python" else "//"
                    with open(os.path.join(d, f), errors="replace") as fh:
                        n = sum(1 for line in fh if line.strip() and
                                not line.strip().startswith(cmt))
                    out[lang] = out.get(lang, 0) + n
        out["total"] = sum(out.values())
        return out

    @property
    def __plugins__(self):
        """Installed plugin packages: entry points of the
        ``veles_amd.plugins`` group (reference ``veles.__plugins__``)."""
        from importlib import metadata
        try:
            eps = metadata.entry_points()
            group = eps.select(group="veles_amd.plugins") \
                if hasattr(eps, "select") else eps.get("veles_amd.plugins",
                                                       ())
        except Exception:  # noqa: BLE001 - broken metadata: no plugins
            return set()
        plugins = set()
        for ep in group:
            try:
                plugins.add(ep.load())
            except Exception:  # noqa: BLE001
                pass
        return plugins

    @staticmethod
    def validate_environment():
        """Interpreter / torch / kernel-library checks before a run
        (reference veles/__init__.py:319-344); returns a list of warnings
        and raises on hard failures."""
        if _sys.version_info < (3, 8):
            raise RuntimeError("veles_amd needs Python >= 3.8")
        warnings = []
        try:
            import torch
        except ImportError:
            raise RuntimeError("veles_amd needs PyTorch (ROCm build)")
        if getattr(torch.version, "hip", None) is None:
            warnings.append("PyTorch is not a ROCm build: CPU device only")
        from veles_amd import ops
        if not ops.available():
            warnings.append("libhvk.so is not built: python -m "
                            "veles_amd.ops.build")
        return warnings

    @staticmethod
    def check_root(allow=None):
        """Refuse to run as root unless allowed (reference ``check_root``,
        veles/__init__.py:346-356); ``VELES_AMD_ALLOW_ROOT=1`` allows."""
        import os
        if allow is None:
            allow = os.environ.get("VELES_AMD_ALLOW_ROOT", "1") == "1"
        if hasattr(os, "geteuid") and os.geteuid() == 0 and not allow:
            raise PermissionError("refusing to run as root "
                                  "(set VELES_AMD_ALLOW_ROOT=1)")


_sys.modules[__name__].__class__ = _VelesModule
