"""HIP-graph capture of the static parts of a training step.

The reference runs every unit's kernels through per-launch Python / OpenCL
calls (``AcceleratedUnit.execute_kernel``, accelerated_units.py:436-455) and
its native runtime plans one arena per workflow (libVeles
src/workflow.cc:44-161); SURVEY §2.6 / §7.4 ask for the MI355X equivalent:
"HIP-graph capture of the static train step".  Here a :class:`GraphSegment`
is a run of consecutive units whose ``run()`` only enqueues device work:

* the forward segment: every forward unit + the evaluator;
* the backward segment: every GD unit (err_input / weight-gradient kernels
  and the fused update launched by the last one).

The unit graph still drives the step (loader, decision, snapshotter, LR
policy stay eager Python between the segments).  For each segment and each
*key* (minibatch class and size, testing flag) the first ``warmup`` passes
run eagerly (lazy allocations, fp8 history priming, split-K workspaces),
the next pass runs inside ``torch.cuda.graph`` capture and is then replayed
once, and every later pass with that key is ONE ``hipGraphLaunch`` - the
segment's units are skipped on the host.  What makes a replay correct:

* kernel arguments that change per step live on the device: the dropout
  seed sequence (``hvk_seed_advance``), the fp8 history slot
  (``hvk_fp8_roll_dev``), the SGD segment table (refreshed by a pre-replay
  hook, ``ParameterStore.refresh_table``, never captured);
* the external inputs of a segment (the loader's minibatch buffers) are
  checked by identity before every replay - a moved buffer drops the graph;
* the device tensors the segment's Arrays point at are recorded at capture
  and re-attached on replay (a unit may alias ``output`` to ``input``
  depending on the key, e.g. dropout on non-TRAIN minibatches), and every
  tensor the graph touches is kept alive as long as the graph;
* host bookkeeping of skipped units runs as replay hooks
  (``ParameterStore.replayed_step``).

A unit class that cannot be captured sets ``graph_safe = False`` (e.g.
stochastic pooling: a torch.Generator seeded from the host per minibatch);
any such unit in a segment keeps that segment eager.  A capture that fails
(an op that synchronises, an unsupported call) re-runs the pass eagerly and
pins that key to eager mode; host state that the discarded capture
advanced (the parameter store's step counters, the fp8 history step) is
restored first (``state_hooks``).  Multi-rank workflows over RCCL can
capture the backward too, collectives included (``engine.dp.graph_backward``:
captured on a one-rank group; at N > 1 "validate" - the first captured
pass of a key is checked against an eager re-run of the same pass on every
rank before the graph is kept, :meth:`GraphSegment._validate`): the
bucketed all-reduces are
enqueued by the GD units in the same order at every rank and RCCL
collectives are stream-capturable, so the graph holds the compute stream's
kernels, each bucket's all-reduce on the process group's stream (forked
from and joined back into the capture by events) and the per-bucket updates
on the update stream - N = 1 and N > 1 replay the same kind of step.  A
backward whose collectives block the host (gloo) or that accumulates
gradients over micro-steps stays eager (``graph_safe`` of the parameter
store).
:func:`suspended` runs passes eagerly for a while (per-bucket timing events
of the instrumented steps cannot be captured).  Disable graphs with
``root.common.engine.graphs = False`` or ``VELES_AMD_GRAPHS=0``.
"""
from __future__ import annotations

import logging
import os

__all__ = ["GraphSegment", "graphs_enabled", "install_step_graphs",
           "suspended"]

_log = logging.getLogger("graphs")

# > 0 while ``suspended()`` is active: every segment runs its passes eagerly
_suspend = 0


class suspended(object):
    """Context manager: segments run eagerly inside it (their graphs are
    kept and replayed again afterwards)."""

    def __enter__(self):
        global _suspend
        _suspend += 1
        return self

    def __exit__(self, *exc):
        global _suspend
        _suspend -= 1
        return False

# the GraphSegment whose capture is in progress (at most one: segments run
# on the main thread, one after the other).  A unit outside it that runs
# while it is open (Unit.do_run -> interrupt_open_capture) would enqueue its
# kernels into the graph - the capture is abandoned instead.
_open_segment = None


def interrupt_open_capture(unit):
    """Called for every unit that is not in a graph segment: abandon an
    open capture (the key runs eagerly from then on, the units captured so
    far re-run eagerly) so that the unit's work is not recorded into it."""
    seg = _open_segment
    if seg is not None and seg.mode == "capture":
        seg.interrupt(unit)


def graphs_enabled():
    from veles_amd.utils.config import root, get
    env = os.environ.get("VELES_AMD_GRAPHS")
    if env is not None:
        return env not in ("0", "false", "False", "")
    return bool(get(root.common.engine.graphs, True))


def _arrays_of(unit):
    from veles_amd.memory import Array
    return [v for v in vars(unit).values() if isinstance(v, Array)]


class _Captured(object):
    __slots__ = ("graph", "key", "inputs", "arrays", "keep")

    def __init__(self, graph, key, inputs):
        self.graph = graph
        self.key = key
        self.inputs = inputs      # [(Array, tensor)] checked before replay
        self.arrays = []          # [(Array, tensor)] re-attached on replay
        self.keep = []            # tensors the graph reads / writes

    def inputs_ok(self):
        for arr, t in self.inputs:
            if arr._devmem is not t:
                return False
        return True

    def restore(self):
        for arr, t in self.arrays:
            if arr._devmem is not t:
                arr.devmem = t
            elif arr._state != 0 and t is not None and t.is_cuda:
                arr._state = 0


def _capture_stream():
    """A capture stream of the kernel library's own (not from torch's
    round-robin stream pool: a stream that a failed capture leaves in the
    invalidated capture state would otherwise come back later as some
    other "new" stream, e.g. a device's compute stream)."""
    import torch
    from veles_amd.ops import _lib
    if _lib.available():
        ptr = _lib.lib().hvk_stream_create()
        if ptr:
            return torch.cuda.ExternalStream(ptr)
    return torch.cuda.Stream()


class _HipCapture(object):
    """Capture context of one HIP graph on a side stream with a private
    memory pool.  Unlike ``torch.cuda.graph`` it restores the stream context
    even when ``capture_end`` raises (a capture broken by a synchronising
    op): the process then continues on the stream it was on."""
    _stream = None
    _retired = []

    def __init__(self, graph):
        self.graph = graph
        self.ctx = None

    def __enter__(self):
        import gc
        import torch
        torch.cuda.synchronize()
        gc.collect()
        torch.cuda.empty_cache()
        if _HipCapture._stream is None:
            _HipCapture._stream = _capture_stream()
        self.ctx = torch.cuda.stream(_HipCapture._stream)
        self.ctx.__enter__()
        try:
            # thread-local: helper threads (thread pool, a process group's
            # watchdog) may keep making stream / event calls meanwhile
            self.graph.capture_begin(capture_error_mode="thread_local")
        except BaseException:
            self._leave()
            self.retire_stream()
            raise
        return self

    def _leave(self):
        ctx, self.ctx = self.ctx, None
        if ctx is not None:
            ctx.__exit__(None, None, None)

    def __exit__(self, *exc):
        from veles_amd.units import _Branches
        ok = False
        try:
            _Branches.join_all()   # unjoined branch streams end the capture
            self.graph.capture_end()
            ok = True
        finally:
            self._leave()
            if not ok:
                self.retire_stream()
                # branch streams forked inside the broken capture joined it:
                # end it on them too (after the origin stream) and fork
                # fresh ones from now on
                _Branches.abandon_capture()
        return False

    @staticmethod
    def retire_stream():
        """A capture that ended in an error can leave its stream in the
        (invalidated) capture state on HIP: the capture is ended on it and
        later captures get a fresh stream - torch pools its streams, so this
        one is handed out again later, e.g. as a Device compute stream, and
        must not still be capturing then.  The thread's pending HIP error is
        drained too, so that the next kernel library launch (which reports
        hipGetLastError) is not charged with it."""
        st, _HipCapture._stream = _HipCapture._stream, None
        if st is not None:
            _HipCapture._retired.append(st)   # never handed out again
        try:
            from veles_amd.ops import _lib
            if _lib.available():
                if st is not None:
                    ended = _lib.lib().hvk_end_stream_capture(st.cuda_stream)
                    _log.info("retired capture stream %#x (capture ended "
                              "here: %d)", st.cuda_stream, ended)
                _lib.lib().hvk_take_last_error()
        except Exception:  # noqa: BLE001 - best effort on an error path
            pass


class GraphSegment(object):
    """Capture / replay of ``units`` (run consecutively, head first).

    key_fn() -> hashable key of the pass, or None to run it eagerly.
    inputs_fn() -> Arrays produced outside the segment that it reads.
    pre_hooks run before every replay or capture (eagerly); replay_hooks
    after every replay, in place of the skipped units' host bookkeeping."""

    MAX_GRAPHS = 8

    def __init__(self, name, units, key_fn, inputs_fn=None, warmup=2,
                 pre_hooks=(), replay_hooks=(), state_hooks=(),
                 validator=None):
        self.name = name
        # validator (optional): checks a key's first captured pass against
        # an eager re-run of the same pass from the same state before the
        # graph is kept (the multi-rank backward, :meth:`_validate`)
        self.validator = validator
        self.validations = []
        self._vsnap = None
        self.units = list(units)
        self.head = self.units[0]
        self.tail = self.units[-1]
        self.key_fn = key_fn
        self.inputs_fn = inputs_fn or (lambda: [])
        self.warmup = warmup
        self.pre_hooks = list(pre_hooks)
        self.replay_hooks = list(replay_hooks)
        # [(save() -> state, restore(state))]: host state a capture pass
        # advances, put back before a failed capture's eager re-run
        self.state_hooks = list(state_hooks)
        self._saved = None
        self.graphs = {}
        self.seen = {}
        self.eager_keys = set()
        self.mode = None
        self.cur = None
        self.ctx = None
        self.pos = 0
        self.captures = 0
        self.replays = 0
        self.failures = 0
        self.safe = all(getattr(u, "graph_safe", True) for u in self.units)
        for u in self.units:
            u.graph_segment_ = self

    def uninstall(self):
        self.drop()
        for u in self.units:
            if getattr(u, "graph_segment_", None) is self:
                u.graph_segment_ = None

    def drop(self, key=None):
        if key is None:
            self.graphs.clear()
        else:
            self.graphs.pop(key, None)

    # -- per-unit dispatch (Unit.do_run) ---------------------------------
    def run_unit(self, unit):
        if unit is self.head:
            self._begin()
        mode = self.mode
        if mode == "replay":
            if unit is self.tail:
                self.mode = None
            return
        self.pos += 1
        try:
            type(unit).run(unit)
        except BaseException as e:
            if mode == "capture":
                self._capture_failed(unit, e)
                return
            self.mode = None
            raise
        if unit is self.tail:
            self._end()

    def _begin(self):
        if self.mode == "capture":  # a previous pass never reached the tail
            self._abort_capture()
        self.mode = "eager"
        self.pos = 0
        if not self.safe or _suspend:
            return
        key = self.key_fn()
        if key is None or key in self.eager_keys:
            return
        for h in self.pre_hooks:
            h()
        g = self.graphs.get(key)
        if g is not None:
            if g.inputs_ok():
                g.graph.replay()
                g.restore()
                for h in self.replay_hooks:
                    h()
                self.replays += 1
                self.mode = "replay"
                return
            _log.info("%s: inputs of graph %r moved, recapturing",
                      self.name, key)
            self.drop(key)
            self.seen[key] = 0
        n = self.seen.get(key, 0)
        if n < self.warmup or len(self.graphs) >= self.MAX_GRAPHS:
            self.seen[key] = n + 1
            return
        graph, ctx = self.new_graph()
        self.cur = _Captured(graph, key, [(a, a._devmem)
                                          for a in self.inputs_fn()])
        self._saved = [save() for save, _ in self.state_hooks]
        v = self.validator
        self._vsnap = v.save() if v is not None and v.wanted() else None
        self.ctx = ctx
        self.ctx.__enter__()
        self.mode = "capture"
        global _open_segment
        _open_segment = self

    @staticmethod
    def new_graph():
        """(graph with .replay(), capture context manager).  Tests swap in a
        host-side recorder; on the GPU it is torch's HIP graph + capture
        on a side stream with a private memory pool."""
        import torch
        graph = torch.cuda.CUDAGraph()
        return graph, _HipCapture(graph)

    def _closed(self):
        global _open_segment
        if _open_segment is self:
            _open_segment = None

    def interrupt(self, unit):
        """a unit outside this segment runs while its capture is open"""
        _log.warning("%s: %s ran while the capture was open; this key runs "
                     "eagerly", self.name, unit)
        self._capture_failed(None, RuntimeError(
            "capture interrupted by %s" % unit))

    def _end(self):
        if self.mode == "capture":
            self._closed()
            cur, ctx = self.cur, self.ctx
            self.cur = self.ctx = None
            try:
                ctx.__exit__(None, None, None)
            except Exception as e:  # noqa: BLE001 - capture_end failed
                self._pin_eager(cur.key, e)
                self.failures += 1
                self.mode = None
                self._restore_state()
                self._rerun_eager(len(self.units))
                return
            saved, self._saved = self._saved, None
            self._record(cur)
            self.graphs[cur.key] = cur
            self.captures += 1
            cur.graph.replay()  # capture records; this pass still has to run
            if self._vsnap is not None:
                self._validate(cur, saved)
        self.mode = None

    def _validate(self, cur, saved):
        """The key's first captured pass against the same pass run eagerly:
        the replayed result is kept aside, the host state (``state_hooks``)
        and the validator's device state are put back to what they were
        before the pass, the units run eagerly (collectives included: every
        rank does the same), and the validator compares the two results and
        agrees on the verdict across ranks.  A mismatch on any rank pins
        the key to eager mode everywhere; the eager pass's state stands
        either way.  Costs one extra pass, once per key."""
        v, snap = self.validator, self._vsnap
        self._vsnap = None
        got = v.result()
        self._saved = saved
        self._restore_state()
        v.restore(snap)
        self.mode = "eager"
        self._rerun_eager(len(self.units))
        ok = bool(v.agree(v.compare(snap, got, v.result())))
        self.validations.append(ok)
        if not ok:
            self.failures += 1
            self._pin_eager(cur.key, RuntimeError(
                "the captured pass differs from the eager pass"))
        else:
            _log.info("%s: captured pass of %r matches the eager pass",
                      self.name, cur.key)

    def _record(self, cur):
        import torch
        from veles_amd import ops
        seen = set()
        for u in self.units:
            for a in _arrays_of(u):
                if id(a) in seen:
                    continue
                seen.add(id(a))
                cur.arrays.append((a, a._devmem))
            for v in vars(u).values():
                if isinstance(v, torch.Tensor):
                    cur.keep.append(v)
        cur.keep.extend(t for _, t in cur.arrays if t is not None)
        # op-level workspaces / cached segment tensors the graph baked in
        cur.keep.extend(ops._WS.values())
        cur.keep.extend(ops._SEG_CACHE.values())

    def _abort_capture(self):
        self._closed()
        ctx, cur = self.ctx, self.cur
        self.ctx = self.cur = None
        if ctx is not None:
            try:
                ctx.__exit__(None, None, None)
            except Exception:  # noqa: BLE001
                pass
        if cur is not None:
            self._pin_eager(cur.key, RuntimeError("capture interrupted"))

    def _capture_failed(self, unit, exc):
        key = self.cur.key if self.cur is not None else None
        self._abort_capture()
        if key is not None:
            self._pin_eager(key, exc)
        self.failures += 1
        # nothing captured has executed: run this pass for real, eagerly
        self.mode = "eager"
        self._restore_state()
        self._rerun_eager(self.pos)
        if unit is self.tail:
            self.mode = None

    def _restore_state(self):
        saved, self._saved = self._saved, None
        if saved is not None:
            for (_, restore), st in zip(self.state_hooks, saved):
                restore(st)

    def _pin_eager(self, key, exc):
        self.eager_keys.add(key)
        self.graphs.pop(key, None)
        _log.warning("%s: graph capture of %r failed (%s); this key runs "
                     "eagerly", self.name, key, exc)

    def _rerun_eager(self, upto):
        for u in self.units[:upto]:
            type(u).run(u)


def _is_chain(units):
    """True when the units run strictly one after another (no other unit
    can run - and be captured - between the head and the tail)."""
    for a, b in zip(units, units[1:]):
        if set(a._links_to) != {b} or set(b._links_from) != {a}:
            return False
    return True


def _full_key(wf):
    ld = wf.loader
    # buffer_parity_: which of a run-ahead loader's two minibatch buffer
    # sets this pass reads (one graph per set: a graph replays the pointers
    # it captured)
    return (int(ld.minibatch_class), int(ld.minibatch_size),
            bool(getattr(wf, "testing", False)),
            int(getattr(ld, "buffer_parity_", 0)))


def install_step_graphs(wf, warmup=2):
    """Attach forward / backward GraphSegments to a StandardWorkflow whose
    device is a GPU.  Returns the installed segments (empty if disabled)."""
    for seg in getattr(wf, "graph_segments_", None) or []:
        seg.uninstall()
    wf.graph_segments_ = []
    dev = getattr(wf, "device", None)
    if not graphs_enabled() or dev is None or not getattr(dev, "is_gpu",
                                                          False):
        return []
    ld = wf.loader
    ev = getattr(wf, "evaluator", None)
    fwd_units = list(wf.forwards) + ([ev] if ev is not None else [])
    if not fwd_units:
        return []

    def inputs():
        out = []
        for name in ("minibatch_data", "minibatch_labels",
                     "minibatch_targets"):
            a = getattr(ld, name, None)
            if a is not None and getattr(a, "_devmem", None) is not None:
                out.append(a)
        return out

    segs = []
    if _is_chain(fwd_units):
        segs.append(GraphSegment("forward", fwd_units,
                                 lambda: _full_key(wf), inputs,
                                 warmup=warmup))
    gds = [g for g in reversed(getattr(wf, "gds", []) or []) if g is not None]
    store = getattr(wf, "param_store_", None)
    if gds and store is not None and _is_chain(gds):
        def bkey():
            if not store.graph_safe():
                return None
            return _full_key(wf)
        segs.append(GraphSegment(
            "backward", gds, bkey, inputs, warmup=warmup,
            pre_hooks=[store.refresh_table],
            replay_hooks=[store.replayed_step],
            state_hooks=[(store.host_state, store.restore_host_state)],
            validator=store.capture_validator()))
    wf.graph_segments_ = segs
    return segs
