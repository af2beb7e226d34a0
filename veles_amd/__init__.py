"""veles_amd - an MI355X-native dataflow deep-learning engine with the
Unit/Workflow programming model of Veles (devbib/veles).

See README.md for the architecture and SURVEY.md for the reference analysis.
"""
__version__ = "0.1.0"
__all__ = ["__version__", "root"]

from veles_amd.utils.config import root  # noqa: E402,F401
