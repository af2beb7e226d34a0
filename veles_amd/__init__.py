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
        from veles_amd.unit_registry import UnitRegistry
        return set(UnitRegistry.units)


_sys.modules[__name__].__class__ = _VelesModule
