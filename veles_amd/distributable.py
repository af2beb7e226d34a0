"""Pickling contract and the distributed data-exchange protocol.

Reference: veles/distributable.py:48-133 (``Pickleable``: attributes whose name
ends with ``_`` are transient and rebuilt by ``init_unpickled``), :136-219
(``Distributable``: thread-safe data hooks with a deadlock warning), :222-281
(``IDistributable``), :284-302 (``TriviallyDistributable``).

In this framework the master/slave roles of the reference become ranks of a
``torch.distributed`` process group (rank 0 = "master").  The five hooks keep
their meaning for the job-farm modes (genetics, ensembles) and for one-off
exchanges (initial-state broadcast); per-step gradient traffic never goes
through them - it is a bucketed RCCL all-reduce (veles_amd/parallel).
"""
from __future__ import annotations

import threading
import time

from veles_amd.mutable import LinkableAttribute
from veles_amd.utils.logger import Logger

__all__ = ["Pickleable", "Distributable", "IDistributable",
           "TriviallyDistributable"]


class Pickleable(Logger):
    """Base of every persistent object.

    * ``foo_`` attributes are not pickled.
    * ``init_unpickled()`` runs after construction AND after unpickling and
      must (re)create every transient attribute.
    """

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.stripped_pickle_ = False
        self.init_unpickled()

    def init_unpickled(self):
        # Logger.init_unpickled creates the logger
        super().init_unpickled()

    @property
    def stripped_pickle(self):
        return getattr(self, "stripped_pickle_", False)

    @stripped_pickle.setter
    def stripped_pickle(self, value):
        self.stripped_pickle_ = value

    def __getstate__(self):
        state = {}
        for k, v in self.__dict__.items():
            if k.endswith("_") and not k.startswith("_lnk_"):
                continue
            if k.startswith("_lnk_"):
                state[k] = v
                continue
            state[k] = v
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        for k in list(state):
            if k.startswith("_lnk_"):
                LinkableAttribute.install(self, k[5:])
        self.init_unpickled()


class IDistributable(object):
    """The five-method data protocol (reference distributable.py:222-281)."""

    def generate_data_for_master(self):
        """Rank k -> rank 0 payload after a job."""

    def generate_data_for_slave(self, slave):
        """Rank 0 -> rank k job payload."""

    def apply_data_from_master(self, data):
        """Consume a rank-0 payload on rank k."""

    def apply_data_from_slave(self, data, slave):
        """Consume a rank-k payload on rank 0."""

    def drop_slave(self, slave):
        """A rank left the group."""


class Distributable(Pickleable):
    DEADLOCK_TIME = 4.0

    def __init__(self, **kwargs):
        self._generate_data_for_slave_threadsafe = kwargs.get(
            "generate_data_for_slave_threadsafe", True)
        self._apply_data_from_slave_threadsafe = kwargs.get(
            "apply_data_from_slave_threadsafe", True)
        super().__init__(**kwargs)

    def init_unpickled(self):
        super().init_unpickled()
        self._data_lock_ = threading.Lock()
        self._data_event_ = threading.Event()
        self._data_event_.set()

    def _locked(self, fn, *args):
        if not self._data_lock_.acquire(timeout=self.DEADLOCK_TIME):
            self.warning("Possible deadlock in %s (waited %.1f s)",
                         fn.__name__, self.DEADLOCK_TIME)
            self._data_lock_.acquire()
        try:
            return fn(*args)
        finally:
            self._data_lock_.release()

    @property
    def has_data_for_slave(self):
        return self._data_event_.is_set()

    @has_data_for_slave.setter
    def has_data_for_slave(self, value):
        if value:
            self._data_event_.set()
        else:
            self._data_event_.clear()

    def wait_for_data_for_slave(self, timeout=None):
        t0 = time.time()
        ok = self._data_event_.wait(timeout)
        if not ok:
            self.warning("Timed out after %.1f s waiting for slave data",
                         time.time() - t0)
        return ok

    def save(self, path):
        import pickle
        with open(path, "wb") as f:
            pickle.dump(self, f, protocol=pickle.HIGHEST_PROTOCOL)

    @staticmethod
    def load(path):
        import pickle
        with open(path, "rb") as f:
            return pickle.load(f)


class TriviallyDistributable(IDistributable):
    def generate_data_for_master(self):
        return None

    def generate_data_for_slave(self, slave):
        return None

    def apply_data_from_master(self, data):
        pass

    def apply_data_from_slave(self, data, slave):
        pass

    def drop_slave(self, slave):
        pass
