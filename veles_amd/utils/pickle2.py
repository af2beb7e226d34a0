"""Pickling helpers (reference veles/pickle2.py:46-111): the best protocol
and an opt-in debugger that names the attribute that cannot be pickled."""
from __future__ import annotations

import pickle

__all__ = ["best_protocol", "dumps", "find_unpicklable"]

best_protocol = pickle.HIGHEST_PROTOCOL


def dumps(obj):
    return pickle.dumps(obj, protocol=best_protocol)


def find_unpicklable(obj, path="obj", seen=None, depth=0):
    """Return the attribute path of the first object that fails to pickle
    (``--debug-pickle``)."""
    seen = seen if seen is not None else set()
    if id(obj) in seen or depth > 12:
        return None
    seen.add(id(obj))
    try:
        pickle.dumps(obj, protocol=best_protocol)
        return None
    except Exception:
        pass
    items = []
    st = getattr(obj, "__getstate__", None)
    try:
        state = st() if st is not None else getattr(obj, "__dict__", None)
    except Exception:
        state = getattr(obj, "__dict__", None)
    if isinstance(state, dict):
        items = list(state.items())
    elif isinstance(obj, (list, tuple)):
        items = list(enumerate(obj))
    elif isinstance(obj, dict):
        items = list(obj.items())
    for k, v in items:
        r = find_unpicklable(v, "%s.%s" % (path, k), seen, depth + 1)
        if r is not None:
            return r
    return path
