"""Diff the unit attributes of two workflow snapshots (reference
veles/scripts/compare_snapshots.py:59-146).

``python -m veles_amd.scripts.compare_snapshots A.pickle.gz B.pickle.gz``
prints, per unit present in both, every attribute whose value differs:
arrays by max |a - b| (and shape / dtype changes), scalars by value.
Snapshots are our own pickles (SnapshotterToFile); never point this at
untrusted files.
"""
from __future__ import annotations

import argparse
import sys

import numpy

__all__ = ["compare", "main"]


def _arr(v):
    t = getattr(v, "devmem", None)
    if t is not None and hasattr(t, "detach"):
        return t.detach().float().cpu().numpy()
    m = getattr(v, "mem", None)
    if m is not None:
        return numpy.asarray(m)
    if hasattr(v, "detach"):
        return v.detach().float().cpu().numpy()
    if isinstance(v, numpy.ndarray):
        return v
    return None


def _units(wf):
    return {u.name: u for u in wf if u is not wf}


def compare(a, b, tolerance=0.0, skip_private=True):
    """[(unit, attribute, description)] of the differences."""
    diffs = []
    ua, ub = _units(a), _units(b)
    for name in sorted(set(ua) ^ set(ub)):
        diffs.append((name, "*", "only in %s" % ("A" if name in ua else "B")))
    for name in sorted(set(ua) & set(ub)):
        da, db = ua[name].__dict__, ub[name].__dict__
        for k in sorted(set(da) | set(db)):
            if skip_private and (k.startswith("_") or k.endswith("_")):
                continue
            if k not in da or k not in db:
                diffs.append((name, k, "missing in %s" %
                              ("B" if k in da else "A")))
                continue
            va, vb = da[k], db[k]
            xa, xb = _arr(va), _arr(vb)
            if xa is not None or xb is not None:
                if xa is None or xb is None:
                    diffs.append((name, k, "array vs non-array"))
                elif xa.shape != xb.shape:
                    diffs.append((name, k, "shape %s vs %s" % (xa.shape,
                                                              xb.shape)))
                elif xa.size:
                    d = float(numpy.max(numpy.abs(
                        xa.astype(numpy.float64) - xb.astype(numpy.float64))))
                    if d > tolerance:
                        diffs.append((name, k, "max |A-B| = %.6g" % d))
                continue
            if isinstance(va, (int, float, str, bool, type(None), tuple,
                               list)):
                try:
                    same = va == vb
                    same = bool(same) if not hasattr(same, "all") else \
                        bool(same.all())
                except Exception:
                    same = False
                if not same:
                    diffs.append((name, k, "%r -> %r" % (va, vb)))
    return diffs


def main(argv=None):
    p = argparse.ArgumentParser(prog="compare_snapshots",
                                description=__doc__.split("\n\n")[0])
    p.add_argument("first")
    p.add_argument("second")
    p.add_argument("-t", "--tolerance", type=float, default=0.0)
    p.add_argument("--all", action="store_true",
                   help="include private / transient attributes")
    args = p.parse_args(argv)
    from veles_amd.snapshotter import SnapshotterToFile
    a = SnapshotterToFile.import_(args.first)
    b = SnapshotterToFile.import_(args.second)
    diffs = compare(a, b, args.tolerance, not args.all)
    for unit, attr, desc in diffs:
        print("%-32s %-32s %s" % (unit, attr, desc))
    print("%d difference(s)" % len(diffs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
