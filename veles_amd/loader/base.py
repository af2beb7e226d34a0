"""Minibatch-serving state machine.

Reference: veles/loader/base.py:118-1181 (``Loader``, ``LoaderMSEMixin``,
``LoaderWithValidationRatio``; serving rules in SURVEY Appendix B item 6):

* samples are laid out TEST | VALID | TRAIN; a pass serves TEST -> VALID ->
  TRAIN; a minibatch never mixes classes (the last one of a class is the
  remainder);
* when the pass ends ``global_offset`` wraps to 0 and only the TRAIN slice is
  reshuffled (``shuffle_limit`` passes at most);
* ``last_minibatch`` = the class ended and nothing is failed/pending;
  ``epoch_ended`` = last minibatch of VALID (of TRAIN when VALID is empty, of
  TEST in test mode);
* padding past ``minibatch_size``: data 0, labels -1, indices -1;
* ``train_ratio`` trims the TRAIN class; failed minibatches are re-served first.

Synchronous data parallelism (replaces the reference's master/slave job
protocol): every rank runs this state machine with the same
seed, so all ranks agree on the global minibatch (class, offset, size) and on
every flag without communication.  Rank r materialises only its contiguous
slice ``[r*B/W, (r+1)*B/W)`` of the global minibatch into its local buffers
(``max_minibatch_size`` is the GLOBAL batch; local buffers hold B/W rows).
``global_minibatch_size`` is what evaluators divide by.
"""
from __future__ import annotations

import time
from collections import defaultdict

import numpy

from veles_amd.distributable import IDistributable
from veles_amd.error import BadFormatError, Bug, MasterSlaveCommunicationError
from veles_amd.memory import Array
from veles_amd.mutable import Bool
from veles_amd.normalization import normalizer as make_normalizer
from veles_amd.prng import random_generator
from veles_amd.units import Unit
from veles_amd.unit_registry import UnitRegistry

__all__ = ["Loader", "LoaderMSEMixin", "LoaderMSE",
           "LoaderWithValidationRatio", "ILoader", "UserLoaderRegistry",
           "TEST", "VALID", "TRAIN", "CLASS_NAME"]

TEST, VALID, TRAIN = 0, 1, 2
CLASS_NAME = ["test", "validation", "train"]
TRIAGE = {"test": TEST, "validation": VALID, "valid": VALID, "train": TRAIN}


class UserLoaderRegistry(UnitRegistry):
    """name -> loader class (reference loader/base.py:83-93)."""
    loaders = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        m = clsdict.get("MAPPING")
        if m:
            UserLoaderRegistry.loaders[m] = cls


class ILoader(object):
    def load_data(self):
        """Fill class_lengths and load / map the dataset."""
        raise NotImplementedError

    def create_minibatch_data(self):
        """Allocate minibatch_data."""
        raise NotImplementedError

    def fill_minibatch(self):
        """Fill minibatch_data (and labels) for minibatch_indices."""
        raise NotImplementedError


class Loader(Unit, ILoader, metaclass=UserLoaderRegistry):
    hide_from_registry = True
    LABEL_DTYPE = numpy.int32
    INDEX_DTYPE = numpy.int32
    exports = ("epoch_ended", "epoch_number", "train_ended", "class_lengths",
               "max_minibatch_size", "minibatch_class", "minibatch_size",
               "minibatch_data", "minibatch_labels", "minibatch_indices",
               "last_minibatch", "has_labels", "total_samples",
               "global_minibatch_size")

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "LOADER")
        self.last_minibatch = Bool(False)
        self.epoch_ended = Bool(False)
        self.train_ended = Bool(False)
        self.test_ended = Bool(False)
        super().__init__(workflow, **kwargs)
        self.prng = kwargs.get("prng", random_generator.get())
        self.testing = bool(kwargs.get("testing", False))
        self.shuffle_limit = kwargs.get("shuffle_limit", numpy.iinfo(
            numpy.uint32).max) if not self.testing else 0
        self.max_minibatch_size = int(kwargs.get("minibatch_size", 100))
        self.class_lengths = [0, 0, 0]
        self.class_end_offsets = [0, 0, 0]
        self._effective_class_end_offsets = [0, 0, 0]
        self._has_labels = False
        self.epoch_number = 0
        self.samples_served = 0
        self.global_offset = 0
        self.minibatch_class = 0
        self.minibatch_offset = 0
        self.minibatch_size = 0
        self.global_minibatch_size = 0
        self.minibatch_data = Array(shallow_pickle=True)
        self.minibatch_indices = Array(shallow_pickle=True)
        self.minibatch_labels = Array(shallow_pickle=True)
        self.raw_minibatch_labels = []
        self.labels_mapping = {}
        self.reversed_labels_mapping = []
        self.failed_minibatches = []
        self.total_failed = 0
        self.shuffled_indices = Array()
        self.normalization_type = kwargs.get("normalization_type", "none")
        self.normalization_parameters = kwargs.get(
            "normalization_parameters", {})
        self.normalizer = make_normalizer(self.normalization_type,
                                          **self.normalization_parameters)
        from veles_amd.utils.config import root, get
        self.train_ratio = float(kwargs.get(
            "train_ratio", get(root.common.loader.train_ratio, 1.0)))
        # data parallel sharding (set by the launcher / process group)
        self.rank = int(kwargs.get("rank", 0))
        self.world_size = int(kwargs.get("world_size", 1))

    def init_unpickled(self):
        super().init_unpickled()
        self.pending_minibatches_ = defaultdict(list)
        self._minibatch_serve_timestamp_ = time.time()
        # sample order before the first shuffle (None: 0..n-1); a validation
        # split extracted by index (loader/labels.py) rearranges it
        self.initial_order_ = None
        self.label_stats = {}
        self.label_distribution_p = {}

    # -- properties ---------------------------------------------------------
    @property
    def has_labels(self):
        return self._has_labels

    @has_labels.setter
    def has_labels(self, value):
        self._has_labels = bool(value)

    @property
    def total_samples(self):
        return sum(self.class_lengths)

    @property
    def effective_class_end_offsets(self):
        return self._effective_class_end_offsets

    @property
    def effective_total_samples(self):
        return self._effective_class_end_offsets[TRAIN]

    @property
    def class_ended(self):
        for off in self.effective_class_end_offsets:
            if self.global_offset == off:
                return True
            if self.global_offset < off:
                return False
        raise Bug("global_offset %d is out of bounds %s" %
                  (self.global_offset, self.class_end_offsets))

    @property
    def local_minibatch_size(self):
        """Rows of this rank's shard of the global minibatch buffer."""
        return -(-self.max_minibatch_size // self.world_size)

    @property
    def pending_minibatches_count(self):
        return sum(len(v) for v in self.pending_minibatches_.values())

    @property
    def unique_labels_count(self):
        return max(len(self.labels_mapping), 1)

    def shard_bounds(self, size):
        """[begin, end) of this rank's rows in a global minibatch of
        ``size`` rows (contiguous split, ceil-sized shards)."""
        per = self.local_minibatch_size
        b = min(size, self.rank * per)
        return b, min(size, b + per)

    # -- lifecycle ----------------------------------------------------------
    def initialize(self, **kwargs):
        if self.testing:
            self.shuffle_limit = 0
            self.global_offset = 0
            del self.failed_minibatches[:]
        self.load_data()
        self.max_minibatch_size = int(kwargs.get("minibatch_size",
                                                 self.max_minibatch_size))
        self._calc_class_end_offsets()
        if not self.restored_from_snapshot or self.testing:
            self.setup_label_stats()
        self.info("Samples number: test: %d, validation: %d, train: %d%s",
                  *(self.class_lengths + [
                      "" if self.train_ratio == 1.0 else
                      " (used %d)" % (self.effective_class_end_offsets[TRAIN] -
                                      self.class_end_offsets[VALID])]))
        n = self.local_minibatch_size
        self.minibatch_labels.reset(
            numpy.zeros(n, dtype=self.LABEL_DTYPE) if self.has_labels
            else None)
        self.minibatch_indices.reset(numpy.zeros(n, dtype=self.INDEX_DTYPE))
        self.raw_minibatch_labels = [None] * n
        self.create_minibatch_data()
        if not self.minibatch_data:
            raise BadFormatError("minibatch_data MUST be initialized in "
                                 "create_minibatch_data()")
        if self.class_lengths[TRAIN] > 0 and not self.restored_from_snapshot:
            self.analyze_dataset()
        elif self.normalizer is not None and self.normalizer.is_initialized:
            self.apply_derived_normalization()
        if not self.restored_from_snapshot or self.testing:
            self.shuffled_indices.reset()
            self.shuffle()
        self.on_initialized(**kwargs)

    @property
    def restored_from_snapshot(self):
        return bool(getattr(self.workflow, "restored_from_snapshot", False))

    def on_initialized(self, **kwargs):
        """Hook: allocate device buffers after the host state is ready."""

    def initial_order(self):
        """Sample order before the first shuffle (int array over all
        samples): the validation split's arrangement or 0..n-1."""
        if self.initial_order_ is not None and \
                len(self.initial_order_) == self.total_samples:
            return numpy.asarray(self.initial_order_, self.INDEX_DTYPE)
        return numpy.arange(self.total_samples, dtype=self.INDEX_DTYPE)

    def class_labels(self):
        """[TEST, VALID, TRAIN] lists of the raw labels of the samples of
        each class, or None when the loader has no per-sample labels to
        analyse (override)."""
        return None

    def setup_label_stats(self):
        """Label mapping, per-class cardinality statistics and the
        distribution check (loader/labels.py)."""
        if not self.has_labels:
            return
        per = self.class_labels()
        if per is None:
            return
        from veles_amd.loader.labels import label_counts, \
            setup_labels_mapping
        setup_labels_mapping(self, [label_counts(c) for c in per],
                             build=self.BUILDS_LABELS_MAPPING)

    # loaders whose labels are raw values (strings, file-derived) get the
    # mapping built from the TRAIN labels; index labels keep theirs
    BUILDS_LABELS_MAPPING = False

    def split_validation(self, labels=None):
        """Move ``validation_ratio`` of the pooled VALID + TRAIN samples
        into VALID by index (stratified per label when ``labels`` - one per
        pooled sample, in sample order - are given; reference
        fullbatch.py:349-433).  ratio <= 0 merges VALID into TRAIN."""
        from veles_amd.loader.labels import random_split, stratified_split
        ratio = getattr(self, "validation_ratio", None)
        if ratio is None:
            return
        if ratio <= 0:
            self.class_lengths[TRAIN] += self.class_lengths[VALID]
            self.class_lengths[VALID] = 0
            return
        if ratio >= 1:
            raise ValueError("validation_ratio must be < 1")
        lo = self.class_lengths[TEST]
        n = self.class_lengths[VALID] + self.class_lengths[TRAIN]
        if labels is not None:
            v, t = stratified_split(labels, ratio, self.prng)
        else:
            v, t = random_split(n, ratio, self.prng)
        order = numpy.arange(lo + n, dtype=self.INDEX_DTYPE)
        order[lo:] = lo + numpy.concatenate(
            [numpy.asarray(v, numpy.int64), numpy.asarray(t, numpy.int64)])
        self.class_lengths[VALID] = len(v)
        self.class_lengths[TRAIN] = len(t)
        self.initial_order_ = order

    def apply_derived_normalization(self):
        """Hook: a loader without TRAIN data that shares an analysed
        normalizer (``derive_from``) prepares to apply it."""

    def run(self):
        self.pending_minibatches_.pop(None, None)
        self.serve_next_minibatch(None)
        self._on_successful_serve()

    # -- serving ------------------------------------------------------------
    def shuffle(self):
        if not self.shuffled_indices:
            self.shuffled_indices.reset(self.initial_order())
        if self.shuffle_limit <= 0 or self.class_lengths[TRAIN] == 0:
            return
        self.shuffle_limit -= 1
        self.shuffled_indices.map_write()
        self.prng.shuffle(self.shuffled_indices.mem[
            self.class_end_offsets[VALID]:])
        self.shuffled_indices.unmap()
        self.on_shuffled()

    def on_shuffled(self):
        """Hook: upload the new permutation to the device."""

    def serve_next_minibatch(self, slave_id):
        try:
            mb = self.failed_minibatches.pop()
        except IndexError:
            mb = self._advance_global_offset()
        offset, size = mb
        self.pending_minibatches_[slave_id].append(mb)
        self.minibatch_offset, self.global_minibatch_size = offset, size
        b, e = self.shard_bounds(size)
        self.minibatch_size = e - b
        self._update_flags()
        if self.fill_indices(offset - size + b, e - b):
            return
        if self.is_master:
            return
        self.fill_minibatch()
        self.normalize_minibatch()
        self.map_minibatch_labels()
        n = self.minibatch_size
        if n < self.local_minibatch_size:
            self.minibatch_data.map_write()
            self.minibatch_data.mem[n:] = 0
            self.minibatch_data.unmap()
            if self.has_labels:
                self.minibatch_labels.map_write()
                self.minibatch_labels.mem[n:] = -1
                self.minibatch_labels.unmap()
            self.minibatch_indices.map_write()
            self.minibatch_indices.mem[n:] = -1
            self.minibatch_indices.unmap()

    def fill_indices(self, start_offset, count):
        """Fill minibatch_indices; return True if minibatch_data was filled
        too (device gather), False if fill_minibatch() must run."""
        self.shuffled_indices.map_read()
        self.minibatch_indices.map_invalidate()
        self.minibatch_indices.mem[:count] = self.shuffled_indices.mem[
            start_offset:start_offset + count]
        self.minibatch_indices.unmap()
        return False

    def normalize_minibatch(self):
        if self.normalizer is not None and self.minibatch_size:
            self.minibatch_data.map_write()
            self.normalizer.normalize(
                self.minibatch_data.mem[:self.minibatch_size])
            self.minibatch_data.unmap()

    def map_minibatch_labels(self):
        if not self.has_labels or not self.labels_mapping:
            return
        self.minibatch_labels.map_write()
        for i, lbl in enumerate(self.raw_minibatch_labels[:self.minibatch_size]):
            self.minibatch_labels.mem[i] = self.labels_mapping[lbl]
        self.minibatch_labels.unmap()

    def analyze_dataset(self):
        """Feed the TRAIN class through the normalizer (reference
        loader/base.py:755-802)."""
        if self.normalizer is None or self.normalizer.stateless:
            if self.normalizer is not None:
                self.normalizer.analyze(None)
            return
        self.analyze_train_data()

    def analyze_train_data(self):
        if self.shuffled_indices.mem is None:
            self.shuffled_indices.reset(self.initial_order())
        start = self.class_end_offsets[VALID]
        end = self.class_end_offsets[TRAIN]
        step = self.local_minibatch_size
        saved = self.minibatch_size
        for off in range(start, end, step):
            n = min(step, end - off)
            self.minibatch_size = n
            self.minibatch_indices.map_invalidate()
            self.minibatch_indices.mem[:n] = self.shuffled_indices.mem[
                off:off + n]
            self.minibatch_indices.unmap()
            self.fill_minibatch()
            self.minibatch_data.map_read()
            self.normalizer.analyze(self.minibatch_data.mem[:n])
        self.minibatch_size = saved

    def class_index_by_sample_index(self, index):
        for ci, off in enumerate(self.effective_class_end_offsets):
            if index < off:
                return ci, off - index
        raise Bug("Could not convert sample index %d to class index" % index)

    def _calc_class_end_offsets(self):
        total = 0
        for i, n in enumerate(self.class_lengths):
            total += int(n)
            self.class_end_offsets[i] = total
        if total == 0:
            raise ValueError("There is no data to serve")
        self._effective_class_end_offsets = list(self.class_end_offsets)
        self._effective_class_end_offsets[TRAIN] -= int(
            (1.0 - self.train_ratio) * self.class_lengths[TRAIN])

    def _update_flags(self):
        last = (self.class_ended and not self.failed_minibatches)
        self.last_minibatch <<= bool(last)
        c = self.minibatch_class
        self.epoch_ended <<= bool(last and (
            c == VALID or
            (c == TEST and self.class_lengths[TRAIN] ==
             self.class_lengths[VALID] == 0) or
            (c == TEST and self.testing) or
            (c == TRAIN and self.class_lengths[VALID] == 0)))

    def _advance_global_offset(self):
        if self.global_offset >= self.effective_total_samples:
            self.global_offset = 0
            self.shuffle()
        self.minibatch_class, remainder = self.class_index_by_sample_index(
            self.global_offset)
        size = min(remainder, self.max_minibatch_size)
        self.global_offset += size
        self.train_ended <<= self.global_offset >= self.effective_total_samples
        self.test_ended <<= self.global_offset >= self.class_end_offsets[TEST]
        return self.global_offset, size

    def _on_successful_serve(self):
        self.samples_served += self.global_minibatch_size
        if self.last_minibatch:
            self.debug("Last minibatch of class %s served in epoch %d",
                       CLASS_NAME[self.minibatch_class].upper(),
                       self.epoch_number)

    # -- job-farm hooks (reference loader/base.py:628-687) -----------------
    def generate_data_for_master(self):
        return True

    def generate_data_for_slave(self, slave):
        sid = getattr(slave, "id", slave)
        self.serve_next_minibatch(sid)
        data = {"indices": self.minibatch_indices.to_numpy()[
            :self.minibatch_size].copy()}
        for attr in ("minibatch_class", "minibatch_size", "minibatch_offset",
                     "epoch_number", "global_minibatch_size"):
            data[attr] = getattr(self, attr)
        self.has_data_for_slave = (not self.class_ended or
                                   bool(self.failed_minibatches))
        return data

    def apply_data_from_master(self, data):
        for attr in ("minibatch_class", "minibatch_size", "minibatch_offset",
                     "epoch_number", "global_minibatch_size"):
            if attr in data:
                setattr(self, attr, data[attr])
        self.last_minibatch <<= False
        self.epoch_ended <<= False
        self.train_ended <<= False
        idx = data["indices"]
        if idx.size != self.minibatch_size:
            raise MasterSlaveCommunicationError("minibatch size mismatch")
        if self.minibatch_offset > len(self.shuffled_indices):
            raise MasterSlaveCommunicationError("minibatch offset overflow")
        self.shuffled_indices.map_write()
        self.shuffled_indices.mem[
            self.minibatch_offset - self.minibatch_size:
            self.minibatch_offset] = idx
        self.shuffled_indices.unmap()

    def apply_data_from_slave(self, data, slave):
        sid = getattr(slave, "id", slave)
        if sid is None:
            return
        try:
            self.minibatch_offset, self.minibatch_size = \
                self.pending_minibatches_[sid].pop()
        except (KeyError, IndexError):
            raise Bug("no pending minibatch for %s" % sid)
        self._on_successful_serve()

    def drop_slave(self, slave):
        sid = getattr(slave, "id", slave)
        if sid in self.pending_minibatches_:
            self.total_failed += 1
            self.failed_minibatches.extend(self.pending_minibatches_[sid])
            del self.pending_minibatches_[sid]
            self.info("Jobs failed: %d/pending: %d",
                      len(self.failed_minibatches),
                      self.pending_minibatches_count)

    # -- results ------------------------------------------------------------
    def get_metric_names(self):
        return {"Total epochs"} if not self.testing else set()

    def get_metric_values(self):
        return {"Total epochs": self.epoch_number} if not self.testing else {}

    def derive_from(self, loader):
        """Share normalization / label mapping with a trained loader
        (reference loader/base.py:249-255)."""
        self.normalization_type = loader.normalization_type
        self.normalization_parameters = loader.normalization_parameters
        self.normalizer = loader.normalizer
        self.labels_mapping = dict(loader.labels_mapping)
        self.reversed_labels_mapping = list(loader.reversed_labels_mapping)


class LoaderMSEMixin(object):
    """Adds regression targets (reference loader/base.py:1034-1155)."""

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.class_targets = Array()
        self.minibatch_targets = Array(shallow_pickle=True)
        self.target_normalization_type = kwargs.get(
            "target_normalization_type", "none")
        self.target_normalizer = make_normalizer(
            self.target_normalization_type,
            **kwargs.get("target_normalization_parameters", {}))


class LoaderMSE(LoaderMSEMixin, Loader):
    hide_from_registry = True


class LoaderWithValidationRatio(Loader):
    """Moves ``validation_ratio`` of TRAIN into VALID at load time."""
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.validation_ratio = kwargs.get("validation_ratio", None)

    def load_data(self):
        """Subclasses fill class_lengths first, then call this: the
        validation set is drawn from the pooled VALID + TRAIN samples by
        index (``split_validation``; stratified when the subclass passes
        its labels)."""
        if self.validation_ratio is None:
            return
        if not self.validation_ratio < 1:
            raise ValueError("validation_ratio must be < 1")
        self.split_validation()
