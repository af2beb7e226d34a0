"""Import a workflow file as a module (reference veles/import_file.py)."""
import importlib.util
import os
import sys


def import_file(path):
    path = os.path.abspath(path)
    name = os.path.splitext(os.path.basename(path))[0]
    d = os.path.dirname(path)
    if d not in sys.path:
        sys.path.insert(0, d)
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod
