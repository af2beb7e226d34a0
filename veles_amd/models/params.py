"""Flat parameter / gradient / momentum storage shared by all layers of a
workflow on one device.

Why flat (MI355X-first):
* ONE fused multi-segment SGD kernel updates every layer per step
  (``hvk_sgd``: reads grad, master, momentum; writes master, momentum and the
  bf16 compute copy) instead of a launch per tensor;
* gradient buckets for the data-parallel all-reduce are contiguous slices of
  the flat fp32 gradient buffer: no pack/unpack copies before RCCL;
* parameters are laid out in REVERSE registration (= reverse forward) order,
  so backward fills the buffer front to back and bucket k can be reduced over
  xGMI while the layers below it are still computing their gradients.

Master weights are float32; the compute copy is the device compute dtype
(bf16 on the MI355X, the master itself on the CPU).
"""
from __future__ import annotations

import logging
import os

import numpy

__all__ = ["ParameterStore", "Param"]


def _cover(segs, total):
    """Extend segments so they tile [0, total) (gaps get lr = 0)."""
    out = []
    pos = 0
    for b, e, lr, d, l1, m in sorted(segs):
        if b > pos:
            out.append((pos, b, 0.0, 0.0, 0.0, 0.0))
        out.append((b, e, lr, d, l1, m))
        pos = e
    if pos < total:
        out.append((pos, total, 0.0, 0.0, 0.0, 0.0))
    return out

_log = logging.getLogger("params")


class Param(object):
    __slots__ = ("owner", "name", "shape", "host", "offset", "size", "master",
                 "lp", "grad", "mom", "gd", "is_bias", "bucket", "host_mom")

    def __init__(self, owner, name, host):
        self.owner = owner
        self.name = name
        self.host = numpy.ascontiguousarray(host, dtype=numpy.float32)
        self.shape = self.host.shape
        self.size = self.host.size
        self.offset = None
        self.master = self.lp = self.grad = self.mom = None
        self.gd = None
        self.is_bias = name == "bias"
        self.bucket = None
        self.host_mom = None


class ParameterStore(object):
    def __init__(self, device, dp=None):
        self.device = device
        self.dp = dp
        self.params = []
        self.finalized = False
        self._ready = set()
        self._works = []
        self._launched = set()
        self.buckets = []
        self._segs = None
        self._solver_segs = None
        self._seg_key = None
        self._seg_table = None
        self.steps = 0
        # micro-steps per optimizer step: > 1 after an elastic shrink keeps
        # the global batch (parallel/launch.py ``shrink``)
        from veles_amd.utils.config import root, get
        self.accumulate = max(1, int(get(
            root.common.engine.dp.accumulate,
            os.environ.get("VELES_AMD_DP_ACCUMULATE", 1))))
        self._accum_count = 0
        # callables run after every applied update (e.g. ZeroFiller masks)
        self.post_update_hooks = []
        # every gradient is WRITTEN once per step by its GD unit (no zeroing
        # pass in the update, no read-modify-write in the FC weight-gradient
        # GEMMs); decided at finalize (see overwrite_ok)
        self.overwrite = False
        self.zero_tail = 0
        # multi-rank: per-bucket updates on a side stream (_overlap_update)
        self._overlap = None
        self._single = None   # single-rank overlapped update (decided once)
        self._tail = None     # single-rank tail-overlapped update (ditto)
        self._tail_evs = None  # branch-stream events of the tail's gradients
        self._span_tables = {}  # (lo, hi) -> segment table of a span update
        self._upd_stream = None
        # gradients are written on branch streams too (weight gradients off
        # the compute stream, gd_conv.py): everything that consumes the
        # gradient buffer then waits for the device's branch streams
        self.branch_grads = False
        self._bucket_tables = {}
        # workgroups of a side-stream bucket update (0: the full grid); one
        # per CU measured best (profiles/dp_overlap_update_r2.md)
        self._upd_blocks = int(os.environ.get("VELES_AMD_DP_UPDATE_BLOCKS",
                                              "256"))
        # wire dtype of the gradient all-reduce: float32, or bfloat16 (half
        # the xGMI bytes; each bucket is cast into a bf16 shadow on the
        # compute stream, reduced, and cast back into the fp32 gradient
        # before the fp32 master update)
        self.grad_dtype = str(get(root.common.engine.dp.grad_dtype,
                                  os.environ.get("VELES_AMD_DP_GRAD_DTYPE",
                                                 "float32")))
        if self.grad_dtype not in ("float32", "bfloat16"):
            raise ValueError("engine.dp.grad_dtype must be float32 or "
                             "bfloat16, not %r" % self.grad_dtype)
        self._shadow = None
        self._pending = {}   # bucket -> (work, shadow view) to cast back
        # exposed-communication instrumentation (bench.py at N > 1): a pair
        # of timing events around the compute stream's wait for the
        # collectives / per-bucket updates, per step
        self.comm_stats = os.environ.get("VELES_AMD_DP_STATS", "0") == "1"
        self._comm_events = []
        # per-bucket timeline of the same instrumented steps: [(t0, [(launch,
        # reduced)] per bucket, end)] events; t0 = the first GD unit's
        # gradients enqueued, launch = the compute stream reaching bucket i's
        # all-reduce, reduced = that all-reduce done (seen from the stream
        # that consumes it), end = the compute stream's join before the next
        # forward.  Eager passes only (graphs.suspended()).
        self._tl = None
        self._timelines = []

    # -- registration -------------------------------------------------------
    def register(self, owner, name, host):
        if self.finalized:
            # late registration (e.g. re-initialize): rebuild
            self.finalized = False
        p = Param(owner, name, host)
        self.params = [q for q in self.params
                       if not (q.owner is owner and q.name == name)]
        self.params.append(p)
        return p

    def find(self, owner, name):
        for p in self.params:
            if p.owner is owner and p.name == name:
                return p
        return None

    def attach_gd(self, param, gd):
        param.gd = gd

    # -- layout -------------------------------------------------------------
    def finalize(self):
        if self.finalized:
            return
        import torch
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        gpu = dev is not None and getattr(dev, "is_gpu", False)
        order = list(reversed(self.params))
        off = 0
        for p in order:
            # keep every parameter 64-element (256 B) aligned for 16-B loads
            off = (off + 63) // 64 * 64
            p.offset = off
            off += p.size
        total = max(off, 1)
        self.total = total
        self.master = torch.zeros(total, dtype=torch.float32, device=tdev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=tdev)
        self.mom = torch.zeros(total, dtype=torch.float32, device=tdev)
        self.mom2 = None  # second solver state (adadelta / rprop), lazily
        lp_dtype = dev.compute_dtype if gpu else torch.float32
        self.lp = torch.zeros(total, dtype=lp_dtype, device=tdev) \
            if lp_dtype != torch.float32 else None
        for p in order:
            sl = slice(p.offset, p.offset + p.size)
            self.master[sl].copy_(torch.from_numpy(p.host.reshape(-1)))
            p.master = self.master[sl].view(p.shape)
            p.grad = self.grad[sl].view(p.shape)
            p.mom = self.mom[sl].view(p.shape)
            p.lp = (self.lp[sl].view(p.shape) if self.lp is not None
                    else p.master)
            if p.host_mom is not None and p.host_mom.size == p.size:
                self.mom[sl].copy_(torch.from_numpy(numpy.ascontiguousarray(
                    p.host_mom, numpy.float32).reshape(-1)))
        if self.dp is not None and self.dp.world_size > 1:
            self.dp.broadcast_(self.master)
        if self.lp is not None:
            self.lp.copy_(self.master)
        self._build_buckets(order)
        self.overwrite = self.overwrite_ok()
        # overwrite mode: the update clears the gradients of the split-K
        # layers (``ZEROED_BY_UPDATE`` GDs, laid out last) after reading them,
        # so those layers need no zeroing launch of their own before their
        # atomics (one pass fused into the update instead of one per layer)
        self.zero_tail = self.total
        if self.overwrite:
            tail = [p.offset for p in order if p.gd is not None and
                    getattr(p.gd, "ZEROED_BY_UPDATE", False)]
            if tail:
                self.zero_tail = min(tail)
        self.finalized = True
        if self.device is not None and getattr(self.device, "fp8", False) \
                and self._multi() and self._amax_sync():
            from veles_amd.ops import fp8
            fp8.registry(self.device.torch_device).dp = self.dp
        for p in order:
            if hasattr(p.owner, "on_params_finalized"):
                p.owner.on_params_finalized()

    def _build_buckets(self, order):
        from veles_amd.utils.config import root, get
        mb = get(root.common.engine.dp.bucket_mb, 32)
        cap = int(mb * (1 << 20) / 4)
        self.buckets = []
        cur = []
        size = 0
        for p in order:
            cur.append(p)
            size += p.size
            if size >= cap:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        # the last bucket can only start reducing when the whole backward
        # is done: keep it to the layers that finish last (AlexNet: conv2 +
        # conv1, 1.4 MB) so conv5..conv3 reduce under their backward
        tail_cap = int(get(root.common.engine.dp.tail_bucket_mb, 2) *
                       (1 << 20) / 4)
        last = self.buckets[-1] if self.buckets else []
        if len(last) > 1:
            tail, size = [], 0
            while len(last) > 1 and size + last[-1].size <= tail_cap:
                size += last[-1].size
                tail.insert(0, last.pop())
            if tail:
                self.buckets.append(tail)
        for i, b in enumerate(self.buckets):
            for p in b:
                p.bucket = i

    def overwrite_ok(self):
        """Gradients may be overwritten instead of accumulated when one step
        is one contribution per parameter (no micro-step accumulation) and
        every GD unit declares it writes its gradients whole
        (``OVERWRITES_GRADS``)."""
        import os as _os
        if _os.environ.get("VELES_AMD_GRAD_OVERWRITE", "1") == "0":
            return False
        gds = [p.gd for p in self.params if p.gd is not None]
        return self.accumulate == 1 and bool(gds) and all(
            getattr(g, "OVERWRITES_GRADS", False) for g in gds)

    def cleared_by_update(self, p):
        """True when the update clears ``p``'s gradient after every step."""
        return (self.overwrite and p is not None and p.offset is not None and
                p.offset >= self.zero_tail)

    def zero_grads(self, params):
        """Zero the gradients of ``params`` (one fill over their span)."""
        ps = [p for p in params if p is not None and p.offset is not None]
        if not ps:
            return
        lo = min(p.offset for p in ps)
        hi = max(p.offset + p.size for p in ps)
        self.grad[lo:hi].zero_()

    def bucket_view(self, i):
        b = self.buckets[i]
        lo = b[0].offset
        hi = b[-1].offset + b[-1].size
        return self.grad[lo:hi]

    # -- step ---------------------------------------------------------------
    def _timing(self):
        """Per-bucket events for this pass (stats mode, eager, GPU)."""
        if not (self.comm_stats and self._multi() and self.master is not None
                and self.master.is_cuda):
            return False
        import torch
        return not torch.cuda.is_current_stream_capturing()

    def _event(self, stream=None):
        import torch
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        return ev

    def grads_ready(self, params):
        """Called by a GD unit once its gradients are enqueued."""
        if not self._ready and self._timing():
            self._tl = (self._event(), {}, {})
        for p in params:
            self._ready.add(id(p))
        if not self._multi():
            if self._single_overlap():
                for i, b in enumerate(self.buckets):
                    if i not in self._launched and \
                            all(id(p) in self._ready for p in b):
                        self._launched.add(i)
                        self._bucket_update(i, None)
            elif self._tail_overlap() and self._tail_evs is None and \
                    all(id(p) in self._ready
                        for b in self.buckets[:-1] for p in b):
                # every gradient but the last bucket's is enqueued: mark the
                # branch streams here, so that the early buckets' update can
                # later wait for exactly these weight gradients (not for the
                # last layers', which it is to run beside)
                import torch
                self._tail_evs = []
                for st in self._grad_streams():
                    ev = torch.cuda.Event()
                    ev.record(st)
                    self._tail_evs.append(ev)
            return
        if self._accum_count + 1 < self.accumulate:
            return
        for i, b in enumerate(self.buckets):
            if i in self._launched:
                continue
            if all(id(p) in self._ready for p in b):
                self._launch_bucket(i)

    def _grad_streams(self):
        """The device's branch streams (units._Branches: a capture that
        failed replaces them, so they are looked up, not remembered)."""
        if not self.branch_grads:
            return []
        from veles_amd.units import _Branches
        return _Branches.streams(self.master.device)

    def _launch_bucket(self, i):
        self._launched.add(i)
        if self.branch_grads and self.master is not None and \
                self.master.is_cuda:
            # the collective (launched from the compute stream) must see the
            # weight gradients written on the branch streams
            import torch
            cur = torch.cuda.current_stream(self.master.device)
            for st in self._grad_streams():
                cur.wait_stream(st)
        if self._tl is not None:
            self._tl[1][i] = self._event()
        view = self.bucket_view(i)
        if self.grad_dtype == "bfloat16":
            import torch
            if self._shadow is None:
                self._shadow = torch.empty(self.total, dtype=torch.bfloat16,
                                           device=self.grad.device)
            lo = self.buckets[i][0].offset
            sh = self._shadow[lo:lo + view.numel()]
            sh.copy_(view)   # compute stream: after the bucket's GD kernels
            work = self.dp.all_reduce_async(sh)
            self._pending[i] = (work, sh)
        else:
            work = self.dp.all_reduce_async(view)
        self._works.append(work)
        if self._overlap_update():
            self._bucket_update(i, work)

    def _finish_bucket(self, i):
        """bf16 wire: cast bucket i's reduced shadow back into the fp32
        gradient (on the current stream, after its collective)."""
        ent = self._pending.pop(i, None)
        if ent is not None:
            ent[0].wait()
            self.bucket_view(i).copy_(ent[1])

    def bucket_layout(self):
        """[(MB, parameter count)] per all-reduce bucket, launch order."""
        return [(round(self.bucket_view(i).numel() * 4 / (1 << 20), 3),
                 len(b)) for i, b in enumerate(self.buckets)]

    def timeline_report(self, reset=True):
        """Per-bucket timeline of the instrumented steps since the last
        report (ms from the first gradient enqueued, mean over steps):
        [{"bucket", "mb", "launch_ms", "reduced_ms"}], plus the compute
        stream's end and the wait exposed after it.  Synchronises."""
        tls = self._timelines
        if reset:
            self._timelines = []
        tls = [t for t in tls if len(t[1]) == len(self.buckets)]
        if not tls:
            return None
        tls[-1][3].synchronize()
        out = []
        for i in range(len(self.buckets)):
            la = [t[0].elapsed_time(t[1][i]) for t in tls]
            rd = [t[0].elapsed_time(t[2][i]) for t in tls if i in t[2]]
            out.append({"bucket": i,
                        "mb": round(self.bucket_view(i).numel() * 4 / 2 ** 20,
                                    2),
                        "launch_ms": round(sum(la) / len(la), 4),
                        "reduced_ms": round(sum(rd) / len(rd), 4)
                        if rd else None})
        end = [t[0].elapsed_time(t[3]) for t in tls]
        last = max((b["launch_ms"] for b in out), default=0.0)
        return {"steps": len(tls), "buckets": out,
                "backward_enqueued_ms": round(last, 4),
                "step_join_ms": round(sum(end) / len(end), 4)}

    def comm_report(self, reset=True):
        """Mean exposed all-reduce wait (ms per step) of the compute stream
        since the last report: the time between the end of this rank's
        backward enqueue and the point where the collectives (and, when
        overlapped, the per-bucket updates) are done.  Synchronises."""
        evs = self._comm_events
        if reset:
            self._comm_events = []
        if not evs:
            return None
        evs[-1][1].synchronize()
        ms = [a.elapsed_time(b) for a, b in evs]
        return {"steps": len(ms), "mean_ms": sum(ms) / len(ms),
                "max_ms": max(ms)}

    # -- per-bucket update overlapped with the backward (multi-rank) ---------
    def _overlap_update(self):
        """Multi-rank plain-SGD steps update each bucket as soon as ITS
        all-reduce is done, on a side stream, while the layers below are
        still in backward (AlexNet: the 58 M classifier parameters, 0.22 ms
        of the 0.24 ms update, leave the critical path).  Off for solver
        segments (adagrad / adadelta / rprop), gradient accumulation and
        ``VELES_AMD_DP_OVERLAP_UPDATE=0``."""
        if self._overlap is None:
            from veles_amd.utils.config import root, get
            mode = os.environ.get(
                "VELES_AMD_DP_OVERLAP_UPDATE",
                "1" if get(root.common.engine.dp.overlap, True) else "0")
            gpu = self.master is not None and self.master.is_cuda
            # a host-blocking wait (gloo on GPU tensors) would stall the
            # backward's launches at every bucket: only when forced
            self._overlap = (
                self._multi() and self.accumulate == 1 and mode != "0" and
                (mode == "force" or not gpu or
                 not getattr(self.dp, "host_blocking_wait", False)))
        if not self._overlap:
            return False
        self._cached_segments()
        return self._solver_segs is None

    def _single_overlap(self):
        """One rank on a GPU, plain SGD, no accumulation: each bucket's
        update runs on the side stream as soon as its GD units are enqueued
        (after their backward-data GEMMs, the last readers of the bf16
        weights in this step), while the lower layers are still in backward.
        Off by default (``root.common.engine.overlap_update = True`` or
        ``VELES_AMD_OVERLAP_UPDATE=1`` turn it on): on AlexNet b1024 the
        side-stream update of the 58 M classifier parameters slowed the
        concurrent weight-gradient GEMMs by more than the 0.22 ms it took
        off the critical path (132.2k -> 129.1k img/s,
        profiles/r3_experiments.md §7)."""
        if self._single is None:
            from veles_amd.utils.config import root, get
            on = os.environ.get(
                "VELES_AMD_OVERLAP_UPDATE",
                "1" if get(root.common.engine.overlap_update, False) else "0")
            gpu = self.master is not None and self.master.is_cuda
            self._single = (on != "0" and gpu and not self._multi() and
                            self.accumulate == 1 and len(self.buckets) > 1)
            if self._single:
                self._cached_segments()
                self._single = self._solver_segs is None
        return self._single

    def _tail_overlap(self):
        """One rank on a GPU, plain SGD, no accumulation: the update of every
        bucket but the last runs on the side stream from the moment the last
        layers' weight gradients are enqueued (their branch streams are not
        waited for), beside them - the memory-bound update of the classifier
        under the MFMA-bound first-layer weight gradient at the end of the
        backward, where the per-bucket overlap above (launched during the
        whole backward) measured slower.  Off by default: AlexNet b2048
        174.8-176.4k img/s with it against 180.1-180.7k without on one box
        (the update's 256 workgroups and HBM traffic slow the persistent
        conv1 weight gradient by more than the 0.22 ms they take off the
        critical path; profiles/r5/ab_tail_update_r5r.log).
        ``root.common.engine.tail_update`` / ``VELES_AMD_TAIL_UPDATE`` (0 / 1).
        """
        if self._tail is None:
            from veles_amd.utils.config import root, get
            on = os.environ.get(
                "VELES_AMD_TAIL_UPDATE",
                "1" if get(root.common.engine.tail_update, False) else "0")
            gpu = self.master is not None and self.master.is_cuda
            self._tail = (on != "0" and gpu and not self._multi() and
                          self.accumulate == 1 and len(self.buckets) > 1 and
                          not self._single_overlap())
            if self._tail:
                self._cached_segments()
                self._tail = self._solver_segs is None
        return self._tail

    def _span_update(self, lo, hi, stream, max_blocks=None):
        """Fused SGD over [lo, hi) of the store on ``stream``."""
        import torch
        from veles_amd import ops
        segs = self._span_segs(lo, hi)
        if not segs:
            return
        zf = True if not self.overwrite else max(0, self.zero_tail - lo)
        if (lo, hi) not in self._span_tables:
            self._span_tables[(lo, hi)] = ops.SegmentTable(self.master.device)
        lp = self.lp[lo:hi] if self.lp is not None else None
        with torch.cuda.stream(stream):
            ops.sgd_update(self.master[lo:hi], self.grad[lo:hi],
                           self.mom[lo:hi], segs, w_lp=lp, zero_grad=zf,
                           table=self._span_tables[(lo, hi)],
                           max_blocks=max_blocks)

    def _span_segs(self, lo, hi):
        """The update segments inside [lo, hi), span-relative."""
        segs = []
        for b, e, lr, d, l1, m in self._cached_segments():
            b, e = max(b, lo), min(e, hi)
            if b < e:
                segs.append((b - lo, e - lo, lr, d, l1, m))
        return segs

    def _bucket_span(self, i):
        """[lo, hi) of bucket i's update: from its first parameter to the
        next bucket's (the last bucket to ``total``), so the spans tile the
        store and stay 16-B aligned for the vector update kernel."""
        lo = self.buckets[i][0].offset
        hi = self.buckets[i + 1][0].offset if i + 1 < len(self.buckets) \
            else self.total
        return lo, hi

    def _bucket_segs(self, i):
        """The update segments inside bucket i's span, span-relative."""
        lo, hi = self._bucket_span(i)
        segs = []
        for b, e, lr, d, l1, m in self._cached_segments():
            b, e = max(b, lo), min(e, hi)
            if b < e:
                segs.append((b - lo, e - lo, lr, d, l1, m))
        return segs

    def _bucket_update(self, i, work):
        import torch
        from veles_amd import ops
        lo, hi = self._bucket_span(i)
        segs = self._bucket_segs(i)
        if not segs and not self.master.is_cuda:
            work.wait()
            self._finish_bucket(i)
            return
        zf = True if not self.overwrite else max(0, self.zero_tail - lo)
        tables = self._bucket_tables
        if i not in tables:
            tables[i] = ops.SegmentTable(self.master.device)
        lp = self.lp[lo:hi] if self.lp is not None else None
        args = (self.master[lo:hi], self.grad[lo:hi], self.mom[lo:hi], segs)
        kw = {"w_lp": lp, "zero_grad": zf, "table": tables[i],
              "max_blocks": self._upd_blocks}
        if not self.master.is_cuda:
            work.wait()
            self._finish_bucket(i)
            ops.sgd_update(*args, **kw)
            return
        if self._upd_stream is None:
            self._upd_stream = torch.cuda.Stream(device=self.master.device)
        if work is None:
            # one rank: the side stream waits for the compute stream (the
            # bucket's GD kernels); joined back in apply()
            self._upd_stream.wait_stream(
                torch.cuda.current_stream(self.master.device))
            for st in self._grad_streams():
                self._upd_stream.wait_stream(st)
        # the side stream waits for this bucket's collective (which itself
        # waited for the compute stream at launch); its writes to the bf16
        # copy cannot race the forward, which finished before that point
        with torch.cuda.stream(self._upd_stream):
            if work is not None:
                work.wait()
                if self._tl is not None:
                    self._tl[2][i] = self._event(self._upd_stream)
                self._finish_bucket(i)
            if segs:
                ops.sgd_update(*args, **kw)

    def all_ready(self):
        return len(self._ready) >= len([p for p in self.params
                                        if p.gd is not None])

    def segments(self):
        segs = []
        for p in sorted(self.params, key=lambda q: q.offset):
            gd = p.gd
            if gd is None:
                continue
            lr, decay, l1, moment = gd.hyper(p.is_bias)
            segs.append((p.offset, p.offset + p.size, lr, decay, l1, moment))
        return segs

    def _solver_of(self, p):
        fn = getattr(p.gd, "solver", None)
        return fn() if fn is not None else (0, 0.0, 0.0)

    def _cached_segments(self):
        key = tuple((id(p.gd), p.gd.hyper(p.is_bias), self._solver_of(p))
                    for p in self.params if p.gd is not None)
        if key != self._seg_key:
            self._seg_key = key
            self._segs = self.segments()
            # cover alignment gaps so every float4 group has a segment
            self._segs = _cover(self._segs, self.total)
            solv = {p.offset: self._solver_of(p) for p in self.params
                    if p.gd is not None}
            self._solver_segs = None
            if any(m for m, _, _ in solv.values()):
                self._solver_segs = [
                    seg + solv.get(seg[0], (0, 0.0, 0.0))
                    for seg in self._segs]
        return self._segs

    def apply(self, gscale=1.0):
        """Wait for the gradient all-reduces, then one fused SGD update."""
        from veles_amd import ops
        self._accum_count += 1
        tail = (not self._multi() and gscale == 1.0 and
                self._tail_evs is not None and self._tail_overlap())
        if tail:
            # the early buckets' update on the side stream, after the compute
            # stream's work so far (the last layers' backward-data / LRN) and
            # the weight gradients marked in grads_ready, beside the last
            # layers' weight gradients still running on the branch streams
            import torch
            cur = torch.cuda.current_stream(self.master.device)
            if self._upd_stream is None:
                self._upd_stream = torch.cuda.Stream(device=self.master.device)
            self._upd_stream.wait_stream(cur)
            for ev in self._tail_evs:
                self._upd_stream.wait_event(ev)
            split = self.buckets[-1][0].offset
            self._span_update(0, split, self._upd_stream,
                              max_blocks=self._upd_blocks)
        self._tail_evs = None
        if self.branch_grads and self.master is not None and \
                self.master.is_cuda:
            # the gradients written off the compute stream are complete
            import torch
            cur = torch.cuda.current_stream(self.master.device)
            for st in self._grad_streams():
                cur.wait_stream(st)
        if self._accum_count < self.accumulate:
            self._ready.clear()
            return False
        overlapped = False
        if not self._multi() and self._single_overlap():
            for i in range(len(self.buckets)):
                if i not in self._launched:
                    self._launched.add(i)
                    self._bucket_update(i, None)
            overlapped = True
            if self._upd_stream is not None:
                import torch
                torch.cuda.current_stream(self.master.device).wait_stream(
                    self._upd_stream)
        elif self._multi():
            import torch
            ev = None
            if self.comm_stats and self.master.is_cuda and \
                    not torch.cuda.is_current_stream_capturing():
                ev = (torch.cuda.Event(enable_timing=True),
                      torch.cuda.Event(enable_timing=True))
                ev[0].record()
            # buckets not launched yet (e.g. params without GD) go now
            for i in range(len(self.buckets)):
                if i not in self._launched:
                    self._launch_bucket(i)
            overlapped = self._overlap_update()
            if not overlapped:
                for w in self._works:
                    w.wait()
                if self._tl is not None:
                    done = self._event()
                    for i in range(len(self.buckets)):
                        self._tl[2].setdefault(i, done)
                for i in list(self._pending):
                    self._finish_bucket(i)
            elif self._upd_stream is not None:
                # every bucket was updated on the side stream: the next
                # forward (compute stream) reads the new weights after it
                import torch
                torch.cuda.current_stream(self.master.device).wait_stream(
                    self._upd_stream)
            if ev is not None and not torch.cuda.is_current_stream_capturing():
                ev[1].record()
                self._comm_events.append(ev)
                del self._comm_events[:-256]
            if self._tl is not None:
                self._timelines.append(self._tl + (self._event(),))
                del self._timelines[:-64]
                self._tl = None
        segs = [] if overlapped else self._cached_segments()
        if segs and self._seg_table is None:
            self._seg_table = ops.SegmentTable(self.master.device)
        if tail:
            # the last bucket here, then the next forward waits for the side
            # stream's update of the others
            import torch
            self._span_update(self.buckets[-1][0].offset, self.total,
                              torch.cuda.current_stream(self.master.device))
            torch.cuda.current_stream(self.master.device).wait_stream(
                self._upd_stream)
        elif overlapped:
            pass  # updated bucket by bucket (``_bucket_update``)
        elif segs and self._solver_segs is not None:
            import torch
            if self.mom2 is None:
                self.mom2 = torch.zeros_like(self.mom)
            ops.solver_update(self.master, self.grad, self.mom, self.mom2,
                              self._solver_segs, w_lp=self.lp,
                              gscale=gscale / self.accumulate,
                              zero_grad=self._zero_arg(),
                              table=self._seg_table)
        elif segs:
            # the fused kernel also zeroes the gradient buffer (unless every
            # gradient is overwritten next step anyway)
            ops.sgd_update(self.master, self.grad, self.mom, segs,
                           w_lp=self.lp, gscale=gscale / self.accumulate,
                           zero_grad=self._zero_arg(),
                           table=self._seg_table)
        elif not self.overwrite:
            self.grad.zero_()
        elif self.zero_tail < self.total:
            self.grad[self.zero_tail:].zero_()
        self._works = []
        self._launched = set()
        self._ready.clear()
        self._accum_count = 0
        self.steps += 1
        if self.device is not None and getattr(self.device, "fp8", False):
            # fp8 delayed scaling: this step's amaxes enter the history (the
            # GLOBAL batch's amaxes at N > 1: ``engine.dp.fp8_amax_sync``)
            from veles_amd.ops import fp8
            fp8.registry(self.device.torch_device).roll(
                dp=self.dp if self._multi() and self._amax_sync() else None)
        for hook in self.post_update_hooks:
            hook()
        return True

    def _amax_sync(self):
        from veles_amd.utils.config import root, get
        return os.environ.get("VELES_AMD_DP_FP8_AMAX_SYNC", "1" if get(
            root.common.engine.dp.fp8_amax_sync, True) else "0") != "0"

    def _zero_arg(self):
        # everything (accumulating GDs) or the split-K tail (overwrite mode)
        return True if not self.overwrite else self.zero_tail

    # -- HIP-graph replay support (veles_amd/graphs.py) ----------------------
    def graph_safe(self):
        """A captured backward may contain the update only when one step is
        one launch sequence: no gradient accumulation over micro-steps, and
        collectives only if they are stream-ordered (RCCL; gloo's block the
        host) and multi-rank capture is not turned off
        (``engine.dp.graph_backward``)."""
        if self.accumulate != 1:
            return False
        if not self._multi():
            return True
        return self.graph_backward_mode() != "eager" and \
            not getattr(self.dp, "host_blocking_wait", True) and \
            not getattr(self, "capture_rejected_", False)

    def graph_backward_mode(self):
        """How a multi-rank backward runs (``engine.dp.graph_backward`` /
        VELES_AMD_DP_GRAPH_BACKWARD): "eager" (0 / False), "capture" (1 /
        True) or "validate" - captured, but each key's first captured pass
        is checked against the same pass run eagerly from the same state on
        every rank, and kept only if all ranks agree (:class:`
        CaptureValidator`).  Default: "capture" on a one-rank (solo) RCCL
        group, "validate" with real peers.  Through a one-rank RCCL group at
        AlexNet b3072 (profiles/r6/n1_path_b3072_r6d.md): dp1 185.7-186.6k
        img/s, eager 181.6-182.5k (-2.2 %; with branch-stream weight
        gradients 175.3-175.7k), captured 185.3-186.1k, validated capture
        186.3-186.5k with the validation passing."""
        from veles_amd.utils.config import root, get
        default = "capture" if getattr(self.dp, "solo", False) else \
            "validate"
        v = os.environ.get("VELES_AMD_DP_GRAPH_BACKWARD")
        if v is None:
            v = get(root.common.engine.dp.graph_backward, default)
        v = str(v).lower()
        if v in ("0", "false", "eager", "none", ""):
            return "eager"
        if v in ("validate", "validated", "auto"):
            return "validate"
        return "capture"

    def capture_validator(self):
        return CaptureValidator(self)

    def _multi(self):
        """Gradients go through collectives (``DataParallel.multi``)."""
        dp = self.dp
        return dp is not None and getattr(dp, "multi", dp.world_size > 1)

    def refresh_table(self):
        """Bring the device segment table up to date BEFORE a replay or a
        capture: the captured update reads rates from the table's fixed
        address, and the upload itself must never be captured."""
        from veles_amd import ops
        segs = self._cached_segments()
        if not segs or self.master is None or not self.master.is_cuda:
            return
        if self._seg_table is None:
            self._seg_table = ops.SegmentTable(self.master.device)
        if self._solver_segs is not None:
            self._seg_table.update(ops._pack_solver_segs(self._solver_segs))
        else:
            self._seg_table.update(ops._pack_sgd_segs(segs))
            # per-bucket tables of the overlapped updates
            for i, tab in self._bucket_tables.items():
                tab.update(ops._pack_sgd_segs(self._bucket_segs(i)))
            for (lo, hi), tab in self._span_tables.items():
                tab.update(ops._pack_sgd_segs(self._span_segs(lo, hi)))

    def replayed_step(self):
        """Host bookkeeping of one update whose kernels ran in a graph."""
        self._works = []
        self._launched = set()
        self._ready.clear()
        self._accum_count = 0
        self.steps += 1
        if self.device is not None and getattr(self.device, "fp8", False):
            from veles_amd.ops import fp8
            fp8.registry(self.device.torch_device).step += 1

    def host_state(self):
        """Host-side step state that ``apply`` advances (saved before a HIP
        graph capture pass, restored if that capture fails and the pass is
        re-run eagerly: graphs.py)."""
        st = {"steps": self.steps, "ready": set(self._ready),
              "works": list(self._works), "launched": set(self._launched),
              "accum": self._accum_count, "pending": dict(self._pending),
              "tail_evs": self._tail_evs}
        if self.device is not None and getattr(self.device, "fp8", False):
            from veles_amd.ops import fp8
            st["fp8_step"] = fp8.registry(self.device.torch_device).step
        return st

    def restore_host_state(self, st):
        self.steps = st["steps"]
        self._ready = set(st["ready"])
        self._works = list(st["works"])
        self._launched = set(st["launched"])
        self._accum_count = st["accum"]
        self._pending = dict(st["pending"])
        # events recorded inside a failed capture must not be waited for
        self._tail_evs = st.get("tail_evs")
        if "fp8_step" in st:
            from veles_amd.ops import fp8
            fp8.registry(self.device.torch_device).step = st["fp8_step"]

    def sync_host(self):
        """Copy master weights back into each Param.host (for snapshots)."""
        for p in self.params:
            if p.master is not None:
                p.host = p.master.detach().float().cpu().numpy().copy()

    def state_dict(self):
        st = {"master": self.master.detach().cpu(),
              "mom": self.mom.detach().cpu(), "steps": self.steps}
        if self.mom2 is not None:
            st["mom2"] = self.mom2.detach().cpu()
        return st

    def load_state_dict(self, st):
        self.master.copy_(st["master"])
        self.mom.copy_(st["mom"])
        if "mom2" in st:
            import torch
            self.mom2 = torch.zeros_like(self.mom)
            self.mom2.copy_(st["mom2"])
        if self.lp is not None:
            self.lp.copy_(self.master)
        self.steps = st.get("steps", 0)


class CaptureValidator(object):
    """Checks a multi-rank backward's first captured pass (graphs.py
    ``GraphSegment._validate``): the device state the backward advances -
    master weights, momentum (and the second solver state), the bf16
    compute copy, the gradient buffer, the fp8 scaler rows and roll counter
    - is snapshotted before the pass and restored for the eager re-run; the
    two passes' weight UPDATES (not the weights: one step moves a weight by
    ~1e-4 of itself, a wrong gradient would hide under a weight tolerance)
    must agree per parameter tensor to ``rtol`` (f32-atomic split-K sums
    make the kernels' results differ in the last bits from run to run), and
    every rank must agree (one MAX all-reduce of a mismatch flag)."""

    rtol = 1e-3

    def __init__(self, store):
        self.store = store

    def wanted(self):
        st = self.store
        return st._multi() and (
            st.graph_backward_mode() == "validate" or
            os.environ.get("VELES_AMD_DP_VALIDATE_CAPTURE", "0") != "0")

    def _fp8(self):
        dev = getattr(self.store, "device", None)
        if dev is None or not getattr(dev, "fp8", False):
            return None
        from veles_amd.ops import fp8
        return fp8.registry(dev.torch_device)

    def save(self):
        st = self.store
        snap = {k: getattr(st, k).clone() for k in
                ("master", "mom", "mom2", "lp", "grad")
                if getattr(st, k, None) is not None}
        reg = self._fp8()
        if reg is not None:
            snap["fp8"] = ([b.clone() for b in reg.blocks],
                           [b.clone() for b in reg.shard_blocks], reg.step)
        return snap

    def restore(self, snap):
        st = self.store
        for k, v in snap.items():
            if k != "fp8":
                getattr(st, k).copy_(v)
        if "fp8" in snap:
            reg = self._fp8()
            blocks, shards, step = snap["fp8"]
            for b, v in zip(reg.blocks, blocks):
                b.copy_(v)
            for b, v in zip(reg.shard_blocks, shards):
                b.copy_(v)
            reg.set_step(step)

    def result(self):
        return self.store.master.clone()

    def compare(self, snap, got, ref):
        """True when the captured pass's update matches the eager pass's,
        tensor by tensor (``forced mismatch``: VELES_AMD_DP_VALIDATE_FAIL_RANK
        = r makes rank r report one, for tests)."""
        import torch
        r = os.environ.get("VELES_AMD_DP_VALIDATE_FAIL_RANK")
        if r is not None and int(r) == int(getattr(self.store.dp, "rank", 0)):
            return False
        before = snap["master"]
        dg, de = got - before, ref - before
        for p in self.store.params:
            if p.offset is None:
                continue
            a = dg[p.offset:p.offset + p.size]
            b = de[p.offset:p.offset + p.size]
            d = float(torch.linalg.vector_norm((a - b).float()))
            n = float(torch.linalg.vector_norm(b.float()))
            if not d <= self.rtol * n + 1e-12:
                _log.warning("captured backward differs from the eager one "
                             "at %s: |d update| %.3g vs |update| %.3g",
                             "%s.%s" % (getattr(p.owner, "name", "?"),
                                        p.name), d, n)
                return False
        return True

    def agree(self, ok):
        """True only if every rank's pass matched.  A rejection turns the
        store's multi-rank backward eager for good (``graph_safe``), and
        with it the branch-stream weight gradients, which measured slower
        in an eager multi-rank step."""
        import torch
        dp = self.store.dp
        if dp is not None and getattr(dp, "world_size", 1) > 1:
            dev = self.store.master.device if dp.backend == "nccl" else "cpu"
            t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float32,
                             device=dev)
            dp.all_reduce_max(t)
            ok = float(t.cpu()[0]) == 0.0
        if not ok:
            self.store.capture_rejected_ = True
        return ok

