"""Whole dataset resident in (device) memory.

Reference: veles/loader/fullbatch.py:78-566 (``FullBatchLoader``: original
data/labels on the device, minibatch by a gather kernel, numpy fallback on
OOM; ``FullBatchLoaderMSE`` for targets).

MI355X design: the dataset stays in HBM as stored (uint8 images stay uint8 -
288 GB per GPU holds ImageNet-scale synthetic sets), the shuffled index
permutation lives on the device, and one ``hvk_fill_minibatch`` launch
gathers the rank's rows, converts uint8 -> bf16 and applies the normalizer's
per-feature affine map (mean / dispersion) in the same pass.  The CPU device
runs the identical op through its float32 reference.
"""
from __future__ import annotations

import numpy

from veles_amd.loader.base import Loader, LoaderMSEMixin, TRAIN, VALID
from veles_amd.memory import Array

__all__ = ["FullBatchLoader", "FullBatchLoaderMSE", "IFullBatchLoader"]


class IFullBatchLoader(object):
    def load_data(self):
        """Fill original_data, original_labels and class_lengths."""


class FullBatchLoader(Loader, IFullBatchLoader):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.original_data = Array()
        self.original_labels = []
        self.validation_ratio = kwargs.get("validation_ratio", None)
        self.on_device = kwargs.get("on_device", True)
        self._affine = None
        # export_affine (StandardWorkflow.link_meandispnorm): serve the raw
        # data and publish the per-feature normalisation as ``mean`` /
        # ``rdisp`` for a separate MeanDispNormalizer unit, as the
        # reference's image loaders do, instead of folding it into the gather
        self.export_affine = kwargs.get("export_affine", False)
        self.mean = Array()
        self.rdisp = Array()

    def init_unpickled(self):
        super().init_unpickled()
        self._dev_labels_ = None
        self._dev_mean_ = None
        self._dev_rdisp_ = None
        self._dev_shuffled_ = None
        # (s, KH, KW, padding) when the first conv asked for its input in
        # space-to-depth layout (request_s2d_input)
        self.s2d_layout_ = None
        self._dev_s2d_affine_ = None
        # run-ahead state (``_runahead``): two output buffer sets, the parity
        # of the one served, the prefetched minibatch (key, parity, event)
        self._ra_bufs_ = None
        self._ra_pending_ = None
        self._ra_stream_ = None
        self._ra_gen_ = 0
        # (generation, (start, count), parity) of the next gather while it
        # waits for the anchor unit (``runahead_anchor_``, set by
        # StandardWorkflow: the first backward unit) to launch it
        self._ra_deferred_ = None
        self.runahead_anchor_ = None
        self.buffer_parity_ = 0
        self.runahead_hits = 0
        self.runahead_misses = 0

    def __getstate__(self):
        st = super().__getstate__()
        # the dataset itself is regenerated / reloaded by load_data()
        st["original_data"] = Array()
        st["original_labels"] = []
        return st

    @property
    def has_labels(self):
        return len(self.original_labels) > 0

    @has_labels.setter
    def has_labels(self, value):
        pass

    @property
    def sample_shape(self):
        return tuple(self.original_data.shape[1:])

    def _torch_dtype_for_minibatch(self):
        import torch
        dev = self.device
        if dev is not None and getattr(dev, "is_gpu", False):
            return dev.compute_dtype
        return torch.float32

    def create_minibatch_data(self):
        import torch
        from veles_amd import ops
        self._ra_bufs_ = None       # run-ahead sets follow the new buffers
        self._ra_pending_ = None
        self._ra_deferred_ = None
        self.buffer_parity_ = 0
        n = self.local_minibatch_size
        dev = self.device
        shape = (n,) + self.sample_shape
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        lay = self.s2d_layout_
        if lay is not None:
            s, KH, KW, padding = lay
            shape = (n,) + ops.s2d_geometry(shape, s, KH, KW, padding)
        t = torch.zeros(shape, dtype=self._torch_dtype_for_minibatch(),
                        device=tdev)
        self.minibatch_data.devmem = t
        self.minibatch_data.s2d_ = None if lay is None else \
            (lay[0], (n,) + self.sample_shape)
        for arr in (self.minibatch_labels, self.minibatch_indices):
            if arr.mem is not None:
                arr.initialize(dev)

    def request_s2d_input(self, s, KH, KW, padding):
        """The first convolution asks for ``minibatch_data`` in its
        space-to-depth layout (ops.S2DImage): the gather then writes the
        normalised s2d image directly (``hvk_fill_minibatch_s2d``) and the
        bf16 NHWC image is never materialised.  Only for uint8 RGB data on
        the GPU with the affine map folded into the gather; returns whether
        the layout is now in effect.  ``minibatch_data.s2d_`` = (s, logical
        NHWC shape) tells every consumer."""
        import torch
        from veles_amd import ops
        dev = self.device
        data = self.original_data.devmem
        if dev is None or not getattr(dev, "is_gpu", False) or \
                data is None or data.dtype != torch.uint8 or \
                data.dim() != 4 or data.shape[3] != 3 or s != 4 or \
                self.export_affine or \
                self._torch_dtype_for_minibatch() != torch.bfloat16:
            return False
        shape = tuple(data.shape[1:])
        feat = int(numpy.prod(shape))
        mean = self._affine[0] if self._affine is not None else \
            numpy.zeros(feat, numpy.float32)
        rdisp = self._affine[1] if self._affine is not None else \
            numpy.ones(feat, numpy.float32)
        pad = tuple(padding)
        self._dev_s2d_affine_ = tuple(
            ops.s2d_affine(torch.from_numpy(numpy.ascontiguousarray(v)),
                           shape, s, KH, KW, pad, f).to(dev.torch_device)
            for v, f in ((mean, 0.0), (rdisp, 1.0)))
        self.s2d_layout_ = (s, KH, KW, pad)
        self.create_minibatch_data()
        return True

    def _apply_validation_ratio(self):
        """``validation_ratio``: VALID = a label-stratified draw from the
        pooled VALID + TRAIN samples, by index (Loader.split_validation)."""
        if self.validation_ratio is None:
            return
        labels = None
        if self.has_labels:
            lo = self.class_lengths[TEST]
            labels = numpy.asarray(self.original_labels)[lo:]
        self.split_validation(labels)

    def class_labels(self):
        """Per class, the labels of its samples: the raw values of the
        mapping (``reversed_labels_mapping``) when there is one, else the
        index labels themselves."""
        lab = numpy.asarray(self.original_labels)
        order = self.initial_order()
        rev = list(self.reversed_labels_mapping or [])
        out, start = [], 0
        for n in self.class_lengths:
            v = lab[order[start:start + n]].tolist()
            if rev:
                v = [rev[i] if 0 <= i < len(rev) else i for i in v]
            out.append(v)
            start += n
        return out

    def class_rows(self, cls):
        """Sample rows of class ``cls`` in the initial order."""
        start = sum(self.class_lengths[:cls])
        return self.initial_order()[start:start + self.class_lengths[cls]]

    def analyze_dataset(self):
        """Analyse the TRAIN slice on the host, then either keep a
        per-feature affine map for the device gather (uint8 / raw data) or
        normalise the whole resident dataset once (reference
        fullbatch.py:336-347)."""
        if self.normalizer is None or self.normalization_type == "none":
            self._affine = None
            return
        data = self.original_data.mem
        rows = numpy.sort(self.class_rows(TRAIN))
        step = 4096
        for i in range(0, len(rows), step):
            self.normalizer.analyze(
                data[rows[i:i + step]].astype(numpy.float32))
        if not self.normalizer.is_initialized:
            self.normalizer.analyze(data[rows[:1]].astype(numpy.float32))
        aff = self.normalizer.affine()
        if aff is not None:
            mean, rdisp = aff
            feat = int(numpy.prod(self.sample_shape))
            mean = numpy.broadcast_to(numpy.asarray(mean, numpy.float32),
                                      (feat,)).copy()
            rdisp = numpy.broadcast_to(numpy.asarray(rdisp, numpy.float32),
                                       (feat,)).copy()
            self._affine = (mean, rdisp)
            self._export_affine()
        else:
            # non-affine normalizer: normalise the resident data once
            d = data.astype(numpy.float32)
            for i in range(0, len(d), step):
                self.normalizer.normalize(d[i:i + step])
            self.original_data.reset(d)
            self._affine = None

    def apply_derived_normalization(self):
        aff = self.normalizer.affine()
        if aff is None:
            d = self.original_data.mem.astype(numpy.float32)
            self.normalizer.normalize(d)
            self.original_data.reset(d)
            self._affine = None
            return
        feat = int(numpy.prod(self.sample_shape))
        self._affine = tuple(numpy.broadcast_to(
            numpy.asarray(a, numpy.float32), (feat,)).copy() for a in aff)
        self._export_affine()

    def _export_affine(self):
        if not self.export_affine or self._affine is None:
            return
        shape = self.sample_shape
        self.mean.reset(self._affine[0].reshape(shape).copy())
        self.rdisp.reset(self._affine[1].reshape(shape).copy())
        self._affine = None  # the gather serves raw samples

    def normalize_minibatch(self):
        pass  # folded into the gather

    def on_initialized(self, **kwargs):
        import torch
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        if self.original_data.devmem is None or \
                self.original_data.devmem.device != tdev:
            self.original_data.initialize(dev)
        lab = numpy.asarray(self.original_labels, dtype=numpy.int32) \
            if self.has_labels else None
        self._dev_labels_ = None if lab is None else torch.from_numpy(
            lab).to(tdev)
        if self._affine is not None:
            self._dev_mean_ = torch.from_numpy(self._affine[0]).to(tdev)
            self._dev_rdisp_ = torch.from_numpy(self._affine[1]).to(tdev)
        self._upload_shuffled()

    def on_shuffled(self):
        self._ra_gen_ += 1   # a prefetch of the old order is stale
        if self._dev_labels_ is not None or self.original_data.devmem is not None:
            self._upload_shuffled()

    def _upload_shuffled(self):
        import torch
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        src = torch.from_numpy(self.shuffled_indices.mem)
        if self._dev_shuffled_ is None or self._dev_shuffled_.device != tdev \
                or self._dev_shuffled_.numel() != src.numel():
            self._dev_shuffled_ = src.to(tdev).clone()
        else:
            self._dev_shuffled_.copy_(src, non_blocking=False)

    def _gather(self, start_offset, count, data_out, labels_out, idx_out):
        from veles_amd import ops
        data = self.original_data.devmem
        if self.s2d_layout_ is not None:
            s, KH, KW, padding = self.s2d_layout_
            ops.fill_minibatch_s2d(
                data, self._dev_shuffled_, start_offset, count, data_out, s,
                KH, KW, padding, *self._dev_s2d_affine_,
                labels=self._dev_labels_, labels_out=labels_out,
                idx_out=idx_out)
            return
        ops.fill_minibatch(
            data, self._dev_shuffled_, start_offset, count, data_out,
            mean=self._dev_mean_, rdisp=self._dev_rdisp_,
            labels=self._dev_labels_, labels_out=labels_out,
            idx_out=idx_out)

    def fill_indices(self, start_offset, count):
        if self._dev_shuffled_ is None:
            self.on_initialized()
        if self._runahead():
            return self._fill_runahead(start_offset, count)
        self._gather(start_offset, count, self.minibatch_data.devmem,
                     self.minibatch_labels.devmem
                     if self.has_labels else None,
                     self.minibatch_indices.devmem)
        return True

    # -- run-ahead (SURVEY §2.6 "loader / compute overlap") ----------------
    def _runahead(self):
        """Double-buffered device gather: the NEXT minibatch's gather runs
        on a side stream into the other buffer set while this step computes
        (GPU, ``root.common.engine.loader_runahead`` / env
        VELES_AMD_LOADER_RUNAHEAD; not for MSE targets).  The step's HIP
        graphs are keyed by ``buffer_parity_`` (graphs.py), one per buffer
        set.  Off by default: on AlexNet b1024 the side-stream gather ran
        beside conv1 (0.50 -> 0.65 ms) and the step was 0.8 % slower
        (144.3k vs 145.4k img/s, profiles/r4/runahead_ab.md); launched at
        the backward instead (_defer_runahead) it measured +0.4 % on one
        box and +0.0 % on another at b3072: the gather, dispatched first,
        holds the CUs until it drains and the GEMM beside it waits
        (profiles/r6/loader_runahead_placement_r6jj.txt)."""
        dev = self.device
        if dev is None or not getattr(dev, "is_gpu", False) or \
                getattr(self, "original_targets", None) is not None:
            return False
        import os
        from veles_amd.utils.config import root, get
        return os.environ.get("VELES_AMD_LOADER_RUNAHEAD", "1" if get(
            root.common.engine.loader_runahead, False) else "0") != "0"

    def _ra_views(self, parity):
        import torch
        if self._ra_bufs_ is None:
            cur = (self.minibatch_data.devmem,
                   self.minibatch_labels.devmem if self.has_labels else None,
                   self.minibatch_indices.devmem)
            other = tuple(None if t is None else torch.empty_like(t)
                          for t in cur)
            self._ra_bufs_ = [cur, other]
            self._ra_stream_ = torch.cuda.Stream(cur[0].device)
        return self._ra_bufs_[parity]

    def _peek_next(self):
        """(start, count) of the minibatch this rank serves next, when it is
        known now without side effects (no reshuffle and no failed
        minibatch in between), else None."""
        if self.failed_minibatches:
            return None
        off = self.global_offset
        if off >= self.effective_total_samples:
            return None
        _, rem = self.class_index_by_sample_index(off)
        size = min(rem, self.max_minibatch_size)
        b, e = self.shard_bounds(size)
        return off + b, e - b

    def _fill_runahead(self, start_offset, count):
        import torch
        self._launch_deferred()   # a gather whose anchor did not run
        cur = torch.cuda.current_stream(self.minibatch_data.devmem.device)
        key = (self._ra_gen_, start_offset, count)
        pend, self._ra_pending_ = self._ra_pending_, None
        if pend is not None and pend[0] == key:
            parity = pend[1]
            cur.wait_event(pend[2])
            self.runahead_hits += 1
        else:
            self.runahead_misses += 1
            parity = self.buffer_parity_ ^ 1 if pend is not None else \
                self.buffer_parity_
            d, lab, idx = self._ra_views(parity)
            if pend is not None:
                cur.wait_event(pend[2])   # the stale prefetch's writes
            self._gather(start_offset, count, d, lab, idx)
        d, lab, idx = self._ra_views(parity)
        self.minibatch_data.devmem = d
        if lab is not None:
            self.minibatch_labels.devmem = lab
        self.minibatch_indices.devmem = idx
        self.buffer_parity_ = parity
        nxt = self._peek_next()
        if nxt is not None and nxt[1] > 0:
            self._ra_deferred_ = (self._ra_gen_, nxt, parity ^ 1)
            if not self._defer_runahead():
                self._launch_deferred()
        return True

    def _defer_runahead(self):
        """Launch the next gather when the backward starts (the anchor unit)
        rather than now.  Now, it runs beside conv1's forward, which streams
        HBM as well and is a persistent kernel (its workgroups wait for the
        gather's); at the backward it runs beside the fully-connected
        GEMMs, which leave LDS and HBM bandwidth to spare.
        ``VELES_AMD_LOADER_RUNAHEAD_AT=fill`` keeps the round-4 placement."""
        import os
        if self.__dict__.get("runahead_anchor_") is None:
            return False
        return os.environ.get("VELES_AMD_LOADER_RUNAHEAD_AT",
                              "backward") != "fill"

    def launch_runahead(self):
        """The anchor unit's ``before_run_`` hook: enqueue the deferred
        gather (not inside an open capture: the next fill launches it)."""
        if self._ra_deferred_ is None:
            return
        import torch
        if torch.cuda.is_current_stream_capturing():
            return
        self._launch_deferred()

    def _launch_deferred(self):
        d, self._ra_deferred_ = self._ra_deferred_, None
        if d is None or d[0] != self._ra_gen_:
            return   # none, or the order changed since (a miss either way)
        import torch
        _, nxt, parity = d
        cur = torch.cuda.current_stream(self.minibatch_data.devmem.device)
        # the other set's readers (the previous step) are all enqueued on
        # the compute stream before this point
        od, ol, oi = self._ra_views(parity)
        free = torch.cuda.Event()
        free.record(cur)
        side = self._ra_stream_
        side.wait_event(free)
        with torch.cuda.stream(side):
            self._gather(nxt[0], nxt[1], od, ol, oi)
            done = torch.cuda.Event()
            done.record(side)
        self._ra_pending_ = ((self._ra_gen_,) + nxt, parity, done)

    def fill_minibatch(self):
        """Host path used by analysis helpers: fill by minibatch_indices."""
        idx = self.minibatch_indices.to_numpy()[:self.minibatch_size]
        self.minibatch_data.map_write()
        self.minibatch_data.mem[:len(idx)] = self.original_data.mem[idx]
        self.minibatch_data.unmap()


class FullBatchLoaderMSE(LoaderMSEMixin, FullBatchLoader):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.original_targets = Array()

    def __getstate__(self):
        st = super().__getstate__()
        st["original_targets"] = Array()
        return st

    def create_minibatch_data(self):
        import torch
        super().create_minibatch_data()
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        n = self.local_minibatch_size
        tshape = (n,) + tuple(self.original_targets.shape[1:])
        self.minibatch_targets.devmem = torch.zeros(
            tshape, dtype=self._torch_dtype_for_minibatch(), device=tdev)

    def on_initialized(self, **kwargs):
        super().on_initialized(**kwargs)
        if self.original_targets.devmem is None:
            self.original_targets.initialize(self.device)

    def fill_indices(self, start_offset, count):
        from veles_amd import ops
        super().fill_indices(start_offset, count)
        ops.fill_minibatch(self.original_targets.devmem, self._dev_shuffled_,
                           start_offset, count, self.minibatch_targets.devmem)
        return True
