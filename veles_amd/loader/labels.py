"""Label bookkeeping of the loaders: the label -> index mapping, per-class
label statistics, the TRAIN-vs-other distribution check, and the
label-stratified extraction of a validation set.

Behaviour of the reference (veles/loader/base.py:925-1018
``_setup_labels_mapping`` / ``_print_label_stats`` /
``_validate_and_fix_other_labels`` / ``_compare_label_distributions``;
veles/loader/fullbatch.py:349-433 ``_resize_validation``;
veles/loader/image.py:623-721 ``_resize_validation_keys``), designed here as
plain functions over label arrays so the full-batch loaders (labels per
sample) and the streaming image loaders (labels per file key) share them.

* ``setup_labels_mapping``: the mapping is built from the TRAIN labels only
  (sorted), unless the loader already has one (a derived / restored
  loader); a TEST / VALID label the training set lacks is an error, a
  training label absent from TEST / VALID is a warning.  Per class it logs
  min / max / mean / sigma of the label cardinalities and keeps them in
  ``loader.label_stats``.
* the distributions of TEST and VALID are compared with TRAIN's by a
  chi-square goodness-of-fit test (scipy); ``loader.label_distribution_p``
  holds the p-values, p <= 0.95 is logged as a warning ("different").
* ``stratified_split``: every label keeps max(1, round(ratio * n)) of its
  samples in VALID (at least one left in TRAIN, else an error); which ones
  is drawn from the loader's PRNG, so ``-r`` seeds reproduce the split.
"""
from __future__ import annotations

from collections import Counter

import numpy

__all__ = ["LoaderError", "label_counts", "setup_labels_mapping",
           "stratified_split", "random_split", "distribution_pvalue"]


class LoaderError(Exception):
    pass


def label_counts(labels):
    """{label: count} of an iterable of labels (None entries ignored)."""
    return dict(Counter(lbl for lbl in labels if lbl is not None))


def _sort_key(v):
    return (str(type(v)), v)


def distribution_pvalue(train_counts, other_counts):
    """Chi-square goodness of fit of ``other``'s label histogram against
    TRAIN's (expected frequencies scaled to other's total); 1.0 when
    either is empty or scipy is absent."""
    keys = sorted(set(train_counts) | set(other_counts), key=_sort_key)
    obs = numpy.array([other_counts.get(k, 0) for k in keys], numpy.float64)
    exp = numpy.array([train_counts.get(k, 0) for k in keys], numpy.float64)
    if obs.sum() == 0 or exp.sum() == 0:
        return 1.0
    exp = exp / exp.sum() * obs.sum()
    keep = exp > 0
    if keep.sum() < 2:
        return 1.0
    try:
        from scipy.stats import chisquare
    except ImportError:  # pragma: no cover - scipy is in the image
        return 1.0
    # renormalise after dropping labels TRAIN lacks (reported separately)
    o, e = obs[keep], exp[keep]
    e = e / e.sum() * o.sum()
    return float(chisquare(o, e)[1])


def _stats_line(counts):
    v = numpy.array(list(counts.values()), numpy.float64)
    keys = list(counts)
    return {"labels": len(v), "samples": int(v.sum()),
            "min": int(v.min()), "min_label": keys[int(v.argmin())],
            "max": int(v.max()), "max_label": keys[int(v.argmax())],
            "mean": float(v.mean()), "std": float(v.std())}


def setup_labels_mapping(loader, counts, names=("test", "validation",
                                                "train"), build=True):
    """``counts`` = [TEST, VALID, TRAIN] label histograms (raw labels).
    Builds (``build``: when the loader has none) / checks
    ``loader.labels_mapping`` and records the statistics."""
    test, valid, train = counts
    if not loader.labels_mapping and build:
        order = sorted(train, key=_sort_key)
        loader.labels_mapping = {k: i for i, k in enumerate(order)}
        loader.reversed_labels_mapping = order
    # labels the other classes may use: the mapping's, else TRAIN's (a
    # loader without TRAIN samples and without a mapping checks nothing)
    known = set(loader.labels_mapping) if loader.labels_mapping else \
        (set(train) if train else None)
    loader.label_stats = {}
    loader.label_distribution_p = {}
    for name, c in zip(names, counts):
        if not c:
            continue
        unknown = set(c) - known if known is not None else ()
        if unknown:
            raise LoaderError("%s labels absent from the training set: %s" %
                              (name, sorted(unknown, key=_sort_key)[:10]))
        missing = known - set(c) if known is not None else ()
        if missing and name != names[2]:
            loader.warning("%d training label(s) never occur in the %s set, "
                           "e.g. %s", len(missing), name,
                           sorted(missing, key=_sort_key)[:5])
        st = _stats_line(c)
        loader.label_stats[name] = st
        spread = st["std"] / st["mean"] if st["mean"] else 0.0
        log = loader.warning if spread > 0.5 else loader.info
        log("%s label cardinalities: %d labels, min %d (%r), max %d (%r), "
            "mean %.1f, sigma %.1f (%d%%)", name, st["labels"], st["min"],
            st["min_label"], st["max"], st["max_label"], st["mean"],
            st["std"], int(round(100 * spread)))
    for name, c in zip(names[:2], (test, valid)):
        if not c or not train:
            continue
        p = distribution_pvalue(train, c)
        loader.label_distribution_p[name] = p
        if p > 0.95:
            loader.info("OK: %s and %s labels have the same distribution "
                        "(chi-square p = %.3f)", names[2], name, p)
        else:
            loader.warning("%s and %s labels have different distributions "
                           "(chi-square p = %.3f)", names[2], name, p)
    return loader.labels_mapping


def stratified_split(labels, ratio, prng):
    """Positions (into ``labels``) that go to VALID and those that stay in
    TRAIN: per label max(1, round(ratio * n)) drawn by ``prng``."""
    labels = list(labels)
    by = {}
    for pos, lbl in enumerate(labels):
        by.setdefault(lbl, []).append(pos)
    valid, train = [], []
    for lbl in sorted(by, key=_sort_key):
        pos = numpy.array(by[lbl], numpy.int64)
        nv = max(int(round(ratio * len(pos))), 1)
        if nv >= len(pos):
            raise LoaderError(
                "label %r has %d sample(s): too few to keep %d in the "
                "validation set and one in the training set" %
                (lbl, len(pos), nv))
        perm = prng.permutation(len(pos))
        valid.extend(pos[perm[:nv]].tolist())
        train.extend(pos[perm[nv:]].tolist())
    return sorted(valid), sorted(train)


def random_split(n, ratio, prng):
    """Unlabelled data: round(ratio * n) random positions go to VALID."""
    nv = int(round(ratio * n))
    perm = prng.permutation(n)
    return sorted(perm[:nv].tolist()), sorted(perm[nv:].tolist())
