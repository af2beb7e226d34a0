"""JSON encoders for results files (reference veles/json_encoders.py:45-67)."""
import json

import numpy


class NumpyJSONEncoder(json.JSONEncoder):
    def default(self, obj):
        if isinstance(obj, numpy.ndarray):
            return obj.tolist()
        if isinstance(obj, numpy.integer):
            return int(obj)
        if isinstance(obj, numpy.floating):
            return float(obj)
        if isinstance(obj, (set, frozenset)):
            return sorted(obj)
        try:
            import torch
            if isinstance(obj, torch.Tensor):
                return obj.detach().cpu().tolist()
        except ImportError:
            pass
        return repr(obj)


class ConfigJSONEncoder(NumpyJSONEncoder):
    def default(self, obj):
        from veles_amd.utils.config import Config, fix_contents
        if isinstance(obj, Config):
            return fix_contents(obj)
        if callable(obj):
            return getattr(obj, "__name__", repr(obj))
        return super().default(obj)
