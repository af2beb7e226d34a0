"""The dataflow graph node.

Behavioural parity with the reference ``Unit`` (reference: veles/units.py:107-913;
firing rules SURVEY Appendix B items 1-3):

* control links ``links_from`` / ``links_to``; a unit runs when EVERY
  ``links_from`` entry has fired since its last run (``open_gate``), unless
  ``ignores_gate``;
* ``gate_block`` (evaluated by the *source*: a blocked destination is not
  notified), ``gate_skip`` (do not ``run()`` but propagate);
* a notification arriving while ``run()`` executes is dropped;
* successors are visited sorted by name; a stopped unit propagates nothing
  (except Containers);
* ``demand()``-ed attributes must be linked before ``initialize()``;
  ``initialize()`` returning True is retried; RNG state captured at the first
  ``initialize`` is restored on re-initialization;
* ``run()`` before ``initialize()`` raises ``NotInitializedError``; ``run()`` after
  ``stop()`` warns (or raises ``RunAfterStopError``).

Execution model (MI355X-first, differs from the reference): the reference
calls a single successor inline and fans out through Twisted worker threads.
Here notifications are processed by a per-thread *trampoline* (an explicit
work queue, FIFO) so a training loop of any length never grows the Python stack,
and all units of a rank run on one host thread that enqueues HIP work on one
compute stream (stream order = data-dependency order, no host sync needed).
``root.common.engine.parallel_fanout = True`` restores thread-pool fan-out.
"""
from __future__ import annotations

import collections
import os
import threading
import time
import uuid

from veles_amd.distributable import Distributable, IDistributable
from veles_amd.error import VelesException
from veles_amd.mutable import Bool, LinkableAttribute, link as _link_attr
from veles_amd.unit_registry import UnitRegistry
from veles_amd.utils.config import root, get, validate_kwargs
from veles_amd.utils.logger import events

__all__ = ["Unit", "TrivialUnit", "Container", "IUnit", "UnitException",
           "NotInitializedError", "RunAfterStopError", "nothing"]


def nothing(*args, **kwargs):
    return None


class UnitException(VelesException):
    def __init__(self, unit, *args):
        super().__init__(*args)
        self.unit = unit


class NotInitializedError(UnitException):
    pass


class RunAfterStopError(UnitException):
    pass


class IUnit(object):
    """Interface every unit implements: initialize(**kwargs) and run()."""

    def initialize(self, **kwargs):
        raise NotImplementedError

    def run(self):
        raise NotImplementedError


_WRAPPED = ("initialize", "run", "stop")


class _Scheduler(object):
    """Per-thread notification trampoline (see module docstring)."""

    _tls = threading.local()

    @classmethod
    def current(cls):
        stack = getattr(cls._tls, "stack", None)
        return stack[-1] if stack else None

    def __init__(self):
        # FIFO: the siblings of a fan-out all run before any of their
        # successors (the single-thread equivalent of the reference running
        # fan-out successors concurrently, units.py:500-505); a LIFO would
        # starve a side branch (e.g. a plotter) behind the training loop
        self.pending = collections.deque()

    def __enter__(self):
        stack = getattr(self._tls, "stack", None)
        if stack is None:
            stack = self._tls.stack = []
        stack.append(self)
        return self

    def __exit__(self, *exc):
        self._tls.stack.pop()
        if not self._tls.stack:
            # the outermost drain is over: branches that never reached a
            # join (dead ends, end_point from one parent) rejoin here
            _Branches.join_all()
        return False

    def drain(self):
        pending = self.pending
        tls = _Branches._tls
        while pending:
            ent = pending.popleft()
            if len(ent) == 3:
                dst, src, br = ent
            else:
                (dst, src), br = ent, None
            tls.br = br
            try:
                dst._check_gate_and_run(src)
            finally:
                tls.br = None


class _Branches(object):
    """Independent branches of a fan-out on HIP streams (SURVEY §2.6
    "intra-process graph concurrency"; the reference runs fan-out successors
    on its thread pool, veles/units.py:485-505).

    With ``root.common.engine.parallel_fanout`` on a GPU workflow, a unit
    whose control links fan out to several runnable successors forks: every
    successor gets a stream of a small per-device pool that first waits on
    the forking stream (an event), and everything that runs downstream of it
    inherits that stream - its kernels run concurrently with the sibling
    branches.  A unit with several control parents (an InputJoiner diamond,
    the join) waits for every parent's stream on the stream the fork came
    from and runs there; its successors continue in the enclosing branch.
    Everything stays on the engine's thread (kernel launches are
    asynchronous: the concurrency is on the device), so a HIP-graph capture
    follows the fork (streams that wait on a captured event join the capture)
    and the join (the capture stream waits on them again).

    A branch context is (stream, enclosing context, fork stream)."""
    _tls = threading.local()
    _pools = {}
    _abandoned = []
    PER_FORK = 4

    @classmethod
    def current(cls):
        return getattr(cls._tls, "br", None)

    @classmethod
    def depth(cls, br):
        d = 0
        while br is not None:
            d, br = d + 1, br[1]
        return d

    @classmethod
    def fork(cls, device, n):
        """n branch contexts forked from the current stream."""
        import torch
        parent = cls.current()
        base = torch.cuda.current_stream(device)
        pool = cls._pools.setdefault(str(device), [])
        d = cls.depth(parent)
        need = (d + 1) * cls.PER_FORK
        while len(pool) < need:
            # the kernel library's own streams, not torch's round-robin pool:
            # a stream that a failed capture leaves in the invalidated state
            # must never come back as some other "new" stream
            # (graphs._capture_stream, abandon_capture)
            from veles_amd.graphs import _capture_stream
            with torch.cuda.device(device):
                pool.append(_capture_stream())
        out = []
        forked = cls._forked()
        for i in range(n):
            st = pool[d * cls.PER_FORK + i % cls.PER_FORK]
            st.wait_stream(base)
            out.append((st, parent, base))
            forked[id(st)] = st
        return out

    @classmethod
    def _forked(cls):
        f = getattr(cls._tls, "forked", None)
        if f is None:
            f = cls._tls.forked = {}
        return f

    @classmethod
    def streams(cls, device):
        """The branch streams of the device's pool (forked so far)."""
        return list(cls._pools.get(str(device), ()))

    @classmethod
    def abandon_capture(cls):
        """After a HIP-graph capture that failed: the branch streams forked
        inside it joined the (invalidated) capture.  End it on every pooled
        branch stream and start new pools, so that no later fork hands out a
        stream still in that state (graphs._HipCapture)."""
        cls._tls.forked = {}
        pools, cls._pools = cls._pools, {}
        cls._abandoned.extend(pools.values())   # never handed out again
        try:
            from veles_amd.ops import _lib
            if not _lib.available():
                return
            for pool in pools.values():
                for st in pool:
                    _lib.lib().hvk_end_stream_capture(st.cuda_stream)
        except Exception:  # noqa: BLE001 - best effort on an error path
            pass

    @classmethod
    def join_all(cls):
        """Make the current stream wait on every branch stream forked since
        the last call.  A join unit only waits on its own parents, so a
        branch that ends anywhere else would otherwise still run while the
        next step's kernels on the compute stream overwrite its inputs, and
        a capture would end with that stream unjoined.  Called when the
        outermost scheduler drain ends and before a HIP graph capture ends
        (graphs._HipCapture)."""
        forked = getattr(cls._tls, "forked", None)
        if not forked:
            return
        import torch
        cls._tls.forked = {}
        cur = torch.cuda.current_stream()
        for st in forked.values():
            if st.cuda_stream != cur.cuda_stream:
                cur.wait_stream(st)


_ROCTX = [None, False]


_GRAPHS = None


def _graphs_mod():
    """veles_amd.graphs, imported on first use (it imports nothing of the
    unit layer at module level, but keeps this module import-light)"""
    global _GRAPHS
    if _GRAPHS is None:
        from veles_amd import graphs
        _GRAPHS = graphs
    return _GRAPHS


def _roctx():
    """torch.cuda.nvtx (roctx on ROCm builds) when unit ranges are enabled
    by ``root.common.trace.roctx`` or ``VELES_AMD_ROCTX=1``: each unit run
    becomes a named range in ``rocprofv3 --marker-trace`` / the torch
    profiler, next to the kernel trace."""
    if not _ROCTX[1]:
        _ROCTX[1] = True
        on = root.common.trace.roctx is True or \
            os.environ.get("VELES_AMD_ROCTX") == "1"
        if on:
            try:
                import torch
                if torch.cuda.is_available():
                    _ROCTX[0] = torch.cuda.nvtx
            except ImportError:
                pass
    return _ROCTX[0]


class Unit(Distributable, IUnit, IDistributable, metaclass=UnitRegistry):
    """General unit of the data-flow model."""

    hide_from_registry = True
    timers = {}
    visible = True

    def __init__(self, workflow, **kwargs):
        self._name = kwargs.get("name")
        self.view_group = kwargs.get("view_group")
        self._demanded = set()
        self._id = str(uuid.uuid4())
        self._links_from = {}
        self._links_to = {}
        self._gate_block = Bool(False)
        self._gate_skip = Bool(False)
        self._ignores_gate = Bool(kwargs.get("ignore_gate", False))
        self._run_calls = 0
        self._remembers_gates = True
        timings = get(root.common.timings, None)
        if isinstance(timings, (set, list, tuple)):
            timings = self.__class__.__name__ in timings
        else:
            timings = bool(timings) if timings is not None else False
        self._timings = kwargs.get("timings", timings)
        self._workflow = None
        super().__init__(**kwargs)
        validate_kwargs(self, **kwargs)
        self.workflow = workflow

    # -- pickling -----------------------------------------------------------
    def init_unpickled(self):
        super().init_unpickled()
        self._gate_lock_ = threading.Lock()
        self._run_lock_ = threading.Lock()
        self._is_initialized_ = False
        self._stopped_ = False
        Unit.timers.setdefault(self._id, 0.0)
        # Instance-level checked wrappers (reference units.py:166-214): a
        # direct ``unit.run()`` / ``unit.initialize()`` is checked and timed;
        # ``super().run()`` inside subclasses resolves on the class.
        d = self.__dict__
        d["initialize"] = self.do_initialize
        d["run"] = self.do_run
        d["stop"] = self.do_stop

    def __getstate__(self):
        state = super().__getstate__()
        for name in _WRAPPED:
            state.pop(name, None)
        if self.stripped_pickle:
            state["_links_from"] = {}
            state["_links_to"] = {}
        return state

    def __repr__(self):
        name = self.__dict__.get("_name")
        if name is not None:
            return '%s.%s "%s"' % (self.__class__.__module__,
                                   self.__class__.__name__, name)
        return object.__repr__(self)

    def __lt__(self, other):
        if not isinstance(other, Unit):
            return NotImplemented
        if self.name != other.name:
            return self.name < other.name
        wf = self.workflow
        if wf is not None and wf is other.workflow and hasattr(wf, "index_of"):
            return wf.index_of(self) < wf.index_of(other)
        return id(self) < id(other)

    # -- identity -----------------------------------------------------------
    @property
    def id(self):
        return self._id

    @property
    def name(self):
        n = self.__dict__.get("_name")
        return n if n is not None else self.__class__.__name__

    @name.setter
    def name(self, value):
        self._name = value

    @property
    def workflow(self):
        return self._workflow

    @workflow.setter
    def workflow(self, value):
        if value is None:
            raise ValueError("Unit must have a hosting Workflow")
        if not hasattr(value, "add_ref"):
            raise TypeError(
                "The first argument of any unit's constructor must be a "
                "workflow (use veles_amd.dummy.DummyWorkflow for a standalone"
                " unit); got %r" % (value,))
        if self._workflow is not None and self._workflow is not value:
            self._workflow.del_ref(self)
        self._workflow = value
        value.add_ref(self)

    @property
    def launcher(self):
        wf = self.workflow
        while wf is not None and not getattr(wf, "is_launcher", False):
            wf = getattr(wf, "workflow", None)
        return wf

    @property
    def is_master(self):
        return bool(getattr(self.workflow, "is_master", False))

    @property
    def is_slave(self):
        return bool(getattr(self.workflow, "is_slave", False))

    @property
    def is_standalone(self):
        return bool(getattr(self.workflow, "is_standalone", True))

    @property
    def interactive(self):
        return bool(getattr(self.workflow, "interactive", False))

    @property
    def device(self):
        return getattr(self.workflow, "device", None)

    @property
    def thread_pool(self):
        return self.workflow.thread_pool

    @property
    def timings(self):
        return self._timings

    # -- gates / links ------------------------------------------------------
    @property
    def demanded(self):
        return self._demanded

    @property
    def links_from(self):
        return self._links_from

    @property
    def links_to(self):
        return self._links_to

    @property
    def links_from_sorted(self):
        return sorted(self._links_from, key=lambda u: u.name)

    @property
    def links_to_sorted(self):
        return sorted(self._links_to, key=lambda u: u.name)

    def _gate_prop(attr):  # noqa: N805 - descriptor factory
        def getter(self):
            return getattr(self, attr)

        def setter(self, value):
            if not isinstance(value, Bool):
                raise TypeError("veles_amd.mutable.Bool type was expected")
            setattr(self, attr, value)
        return property(getter, setter)

    gate_block = _gate_prop("_gate_block")
    gate_skip = _gate_prop("_gate_skip")
    ignores_gate = _gate_prop("_ignores_gate")
    del _gate_prop

    @property
    def stopped(self):
        return self._stopped_

    @stopped.setter
    def stopped(self, value):
        self._stopped_ = bool(value)

    @property
    def is_initialized(self):
        return self._is_initialized_

    @property
    def run_was_called(self):
        return self._run_calls > 0

    @property
    def total_run_time(self):
        return Unit.timers.get(self._id, 0.0)

    @property
    def average_run_time(self):
        return self.total_run_time / self._run_calls if self._run_calls else 0

    def link_from(self, *args):
        with self._gate_lock_:
            for src in args:
                if src is self:
                    raise ValueError("A unit cannot link from itself")
                self._links_from[src] = False
                src._links_to[self] = False
        return self

    def unlink_from(self, *args):
        with self._gate_lock_:
            for src in args:
                src._links_to.pop(self, None)
                self._links_from.pop(src, None)
        return self

    def unlink_before(self):
        with self._gate_lock_:
            for src in list(self._links_from):
                src._links_to.pop(self, None)
            self._links_from.clear()
        return self

    def unlink_after(self):
        with self._gate_lock_:
            for dst in list(self._links_to):
                dst._links_from.pop(self, None)
            self._links_to.clear()
        return self

    def unlink_all(self):
        self.unlink_before()
        self.unlink_after()
        return self

    def insert_after(self, *chain):
        """Insert a chain of units between this unit and its successors."""
        successors = list(self._links_to)
        self.unlink_after()
        chain[0].link_from(self)
        for dst in successors:
            dst.link_from(chain[-1])
        return self

    def derefed_links_to(self):
        return sorted(self._links_to)

    def derefed_links_from(self):
        return sorted(self._links_from)

    def open_gate(self, *srcs):
        if self._ignores_gate:
            return True
        with self._gate_lock_:
            lf = self._links_from
            if not lf:
                return True
            for src in srcs:
                if src in lf:
                    lf[src] = True
            if not all(lf.values()):
                return False
            self._close_gate()
        return True

    def _close_gate(self):
        for src in self._links_from:
            self._links_from[src] = False
            if self in src._links_to:
                src._links_to[self] = False

    def close_gate(self):
        with self._gate_lock_:
            self._close_gate()

    def close_upstream(self):
        for dst in self._links_to:
            if self in dst._links_from:
                dst._links_from[self] = False
        return self

    # -- data links ---------------------------------------------------------
    @staticmethod
    def is_immutable(value):
        return isinstance(value, (tuple, int, float, complex, bool, str,
                                  bytes, type(None)))

    def link_attrs(self, other, *args, **kwargs):
        """``self.mine`` := live reference to ``other.yours``.

        Immutable values get a LinkableAttribute (live read); mutable objects
        (Arrays, lists, tensors) are shared by reference.
        """
        two_way = kwargs.get("two_way", False)
        for arg in args:
            if (isinstance(arg, tuple) and len(arg) == 2 and
                    isinstance(arg[0], str) and isinstance(arg[1], str)):
                mine, yours = arg
            elif isinstance(arg, str):
                mine = yours = arg
            else:
                raise TypeError(repr(arg) + " is not a valid attributes pair")
            self._link_attr(other, mine, yours, two_way)
        return self

    def _link_attr(self, other, mine, yours, two_way):
        if isinstance(other, Container) and not hasattr(other, yours):
            setattr(other, yours, False)
        try:
            attr = getattr(other, yours)
        except AttributeError:
            self.error("Unable to link %s.%s to %s.%s", other, yours, self,
                       mine)
            raise
        if Unit.is_immutable(attr):
            _link_attr(self, mine, other, yours, two_way=two_way)
        else:
            if mine in type(self).__dict__ and isinstance(
                    type(self).__dict__[mine], LinkableAttribute):
                self.__dict__.pop("_lnk_" + mine, None)
            setattr(self, mine, attr)

    def demand(self, *args):
        for attr in args:
            if attr in self._demanded:
                continue
            if getattr(self, attr, None) is not None:
                self._demanded.add(attr)
                continue
            setattr(self, attr, None)
            self._demanded.add(attr)

    def undemand(self, *args):
        for attr in args:
            self._demanded.discard(attr)

    # -- lifecycle wrappers -------------------------------------------------
    def initialize(self, **kwargs):
        """Override in subclasses.  Return True to be retried later."""
        return None

    def run(self):
        """Override in subclasses."""

    def stop(self):
        """Interrupt a blocking run() (default: nothing)."""

    def do_initialize(self, **kwargs):
        """Checked initialize: demanded attrs, reproducible RNG, retry flag."""
        validate_kwargs(self, **kwargs)
        for attr in sorted(self._demanded):
            if getattr(self, attr, None) is None:
                raise AttributeError(
                    "Attribute %s of unit %s is not linked" % (attr, self))
        saved = self.__dict__.get("_saved_rg_states")
        restore = {}
        from veles_amd.prng.random_generator import RandomGenerator
        for key, value in list(self.__dict__.items()):
            if isinstance(value, RandomGenerator):
                if saved is None:
                    saved = {}
                if key not in saved:
                    saved[key] = value.state
                else:
                    restore[key] = value.state
                    value.state = saved[key]
        if saved:
            self._saved_rg_states = saved
        if not getattr(type(self), "DISABLE_INTERFACE_VERIFICATION", False):
            from veles_amd.verified import Verified
            Verified.verify_interface(self, IUnit)
        retry = type(self).initialize(self, **kwargs)
        for key, st in restore.items():
            getattr(self, key).state = st
        if not retry:
            self._is_initialized_ = True
        return retry

    def do_run(self):
        """Checked, timed run()."""
        if not self._is_initialized_:
            raise NotInitializedError(self, "%s is not initialized" % self)
        if self._stopped_:
            from veles_amd.thread_pool import ThreadPool
            if ThreadPool.interrupted:
                for unit in self._links_from:
                    unit.gate_block <<= True
                return
            if root.common.exceptions.run_after_stop is True:
                raise RunAfterStopError(
                    self, "%s's run() was called after stop()" % self)
            self.warning("run() was called after stop(); check the control "
                         "flow links of %s", self.workflow)
            return
        t0 = time.perf_counter()
        if events.enabled:
            events.record(self.name, "begin")
        rng = _roctx()
        # work other units enqueue at this point of the step (the loader's
        # run-ahead gather at the first backward unit, loader/fullbatch.py)
        hooks = self.__dict__.get("before_run_")
        if hooks:
            for h in hooks:
                h()
        # a unit inside a captured HIP-graph segment (veles_amd/graphs.py)
        # is dispatched by the segment: eager, captured or replayed
        seg = self.__dict__.get("graph_segment_")
        if seg is None and _graphs_mod()._open_segment is not None:
            _graphs_mod().interrupt_open_capture(self)
        body = type(self).run if seg is None else seg.run_unit
        if rng is not None:
            rng.range_push(self.name)
            try:
                body(self)
            finally:
                rng.range_pop()
        else:
            body(self)
        dt = time.perf_counter() - t0
        if events.enabled:
            events.record(self.name, "end")
        Unit.timers[self._id] = Unit.timers.get(self._id, 0.0) + dt
        self._run_calls += 1
        if self._timings:
            self.debug("run took %.6f sec", dt)
        if root.common.trace.run is True:
            self.debug("Call #%d finished @%s", self._run_calls,
                       threading.current_thread().name)

    def do_stop(self):
        type(self).stop(self)
        self._stopped_ = True

    def initialize_dependent(self):
        for unit in self.dependent_units():
            unit.do_initialize()

    # -- firing -------------------------------------------------------------
    def run_dependent(self):
        if self._stopped_ and not isinstance(self, Container):
            return
        links = self.links_to_sorted
        blocks = [bool(dst._gate_block) for dst in links]
        targets = [dst for dst, b in zip(links, blocks)
                   if not b and not dst._gate_block]
        if not targets:
            return
        if root.common.trace.run is True:
            for dst in targets:
                self.debug("%s -> %s @%s", self, dst,
                           threading.current_thread().name)
        brs = None
        if len(targets) > 1 and get(root.common.engine.parallel_fanout,
                                    False) is True:
            dev = self._branch_device()
            if dev is None:
                for dst in targets:
                    self.thread_pool.callInThread(_run_in_pool, dst, self)
                return
            brs = _Branches.fork(dev, len(targets))
        if brs is None:
            brs = [_Branches.current()] * len(targets)
        sched = _Scheduler.current()
        if sched is None:
            with _Scheduler() as sched:
                for dst, br in zip(targets, brs):
                    sched.pending.append((dst, self, br))
                sched.drain()
        else:
            for dst, br in zip(targets, brs):
                sched.pending.append((dst, self, br))

    def _branch_device(self):
        """The torch device of a GPU workflow with engine.branch_streams
        (default on), else None (fan-out on the thread pool)."""
        if get(root.common.engine.branch_streams, True) is not True:
            return None
        wf = self.workflow
        while wf is not None and getattr(wf, "device", None) is None:
            wf = getattr(wf, "workflow", None)
        dev = getattr(wf, "device", None) if wf is not None else None
        if dev is None or not getattr(dev, "is_gpu", False):
            return None
        return dev.torch_device

    def _check_gate_and_run(self, src):
        if not self.open_gate(src):
            return
        wf = self.workflow
        pool = getattr(wf, "_thread_pool_", None) if wf is not None else None
        if pool is not None and pool.failure is not None:
            return
        br = _Branches.current()
        if not self._gate_skip:
            if not self._run_lock_.acquire(False):
                return
            try:
                if br is None:
                    self.ran_on_ = None
                    self.do_run()
                else:
                    br = self._run_on_branch(br)
            finally:
                self._run_lock_.release()
        if br is not _Branches.current():
            # a join: the successors continue in the enclosing branch
            _Branches._tls.br = br
            try:
                self.run_dependent()
            finally:
                _Branches._tls.br = None
            return
        self.run_dependent()

    def _run_on_branch(self, br):
        """do_run() on branch br's stream; a unit with several control
        parents joins them on the fork stream first.  Returns the branch
        context its successors inherit."""
        import torch
        stream, parent, base = br
        if len(self._links_from) > 1:
            for u in self._links_from:
                s = u.__dict__.get("ran_on_")
                if s is not None and s is not base:
                    base.wait_stream(s)
            stream, br = base, parent
        with torch.cuda.stream(stream):
            self.do_run()
        self.ran_on_ = stream
        return br

    def dependent_units(self, with_open_gate=False):
        """BFS over links_to, children sorted by name."""
        yield self
        visited = {self}
        walk = [(child, self) for child in sorted(self._links_to)]
        while walk:
            node, parent = walk.pop(0)
            if node in visited or (with_open_gate and
                                   not node.open_gate(parent)):
                continue
            yield node
            visited.add(node)
            walk.extend((c, node) for c in sorted(node._links_to))

    def describe(self):
        return ("Unit: %s\nClass: %s.%s\nIncoming: %s\nOutgoing: %s" % (
            self.name, type(self).__module__, type(self).__name__,
            [u.name for u in self.links_from_sorted],
            [u.name for u in self.links_to_sorted]))


def _run_in_pool(dst, src):
    with _Scheduler() as sched:
        sched.pending.append((dst, src))
        sched.drain()


class TrivialUnit(Unit):
    """A unit that does nothing (used for tests and as a graph placeholder)."""

    def initialize(self, **kwargs):
        pass

    def run(self):
        pass


class Container(Unit):
    """Marker base: a unit holding other units (Workflow)."""

    hide_from_registry = True
