"""Pickling helpers (reference veles/pickle2.py:46-111): the best protocol
and an opt-in debugger that names the attribute that cannot be pickled."""
from __future__ import annotations

import logging
import pickle
import sys

__all__ = ["best_protocol", "dumps", "find_unpicklable",
           "setup_pickle_debug", "teardown_pickle_debug"]

best_protocol = pickle.HIGHEST_PROTOCOL
# the unwrapped serializer (find_unpicklable must not recurse into the
# --debug-pickle wrappers)
_raw_dumps = pickle.dumps


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
        _raw_dumps(obj, protocol=best_protocol)
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


_saved = None


def setup_pickle_debug(interactive=None):
    """``--debug-pickle`` (reference veles/pickle2.py:66-111): every
    ``pickle.dump`` / ``pickle.dumps`` that fails names the attribute path
    of the object that cannot be pickled (``find_unpicklable``) in the
    raised PicklingError and in the log; on a terminal (or with
    ``interactive=True``) it also opens the post-mortem debugger there.
    Unpickling failures are reported the same way."""
    global _saved
    if _saved is not None:
        return
    _saved = (pickle.dump, pickle.dumps, pickle.load, pickle.loads)
    log = logging.getLogger("pickle2")

    def _debug(exc):
        if interactive if interactive is not None else sys.stdin.isatty():
            import pdb
            pdb.post_mortem(exc.__traceback__)

    def wrap_save(fn):
        def save(obj, *args, **kwargs):
            try:
                return fn(obj, *args, **kwargs)
            except Exception as e:  # noqa: BLE001
                path = find_unpicklable(obj)
                msg = "pickling failed at %s (%s: %s)" % (
                    path, type(e).__name__, e)
                log.error(msg)
                _debug(e)
                raise pickle.PicklingError(msg) from e
        return save

    def wrap_load(fn):
        def load(*args, **kwargs):
            try:
                return fn(*args, **kwargs)
            except Exception as e:  # noqa: BLE001
                log.error("unpickling failed (%s: %s)", type(e).__name__, e)
                _debug(e)
                raise
        return load

    pickle.dump = wrap_save(_saved[0])
    pickle.dumps = wrap_save(_saved[1])
    pickle.load = wrap_load(_saved[2])
    pickle.loads = wrap_load(_saved[3])


def teardown_pickle_debug():
    global _saved
    if _saved is not None:
        pickle.dump, pickle.dumps, pickle.load, pickle.loads = _saved
        _saved = None
