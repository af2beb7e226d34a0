"""Workflow snapshots and exact resume.

Reference: veles/snapshotter.py:82-535 (``SnapshotterBase`` rate-limited by
``interval`` runs and ``time_interval`` seconds; ``SnapshotterToFile`` naming
``{prefix}_{suffix}.{protocol}.pickle[.ext]`` + ``{prefix}_current...`` symlink,
codecs none/snappy/gz/bz2/xz; ``SnapshotterToDB`` (ODBC); ``import_``).

Kept: file naming, codecs (snappy is not available on this image and maps to
gz with a warning), the symlink, the size warning with the top-5 units, the
final snapshot on ``stop()``.  The DB sink is SQLite (stdlib) with the same
(prefix, suffix, timestamp, blob) shape.  Data-parallel: only rank 0 writes,
after a barrier, at a point where every replica holds identical weights.
Device tensors are pulled to the host by the units' ``__getstate__``; the
HIP RNG / torch generator states are captured via RandomGenerator.state.
"""
from __future__ import annotations

import bz2
import gzip
import io
import lzma
import logging
import os
import pickle
import sqlite3
import time

from veles_amd.mutable import Bool
from veles_amd.units import Unit
from veles_amd.utils.config import root, get

__all__ = ["SnapshotterBase", "SnapshotterToFile", "SnapshotterToDB",
           "SnapshotterRegistry"]

PROTOCOL = pickle.HIGHEST_PROTOCOL


class SnapshotterRegistry(type(Unit)):
    snapshotters = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        m = clsdict.get("MAPPING")
        if m:
            SnapshotterRegistry.snapshotters[m] = cls


def _rank():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:
        pass
    return int(os.environ.get("RANK", "0"))


class SnapshotterBase(Unit, metaclass=SnapshotterRegistry):
    hide_from_registry = True
    SIZE_WARNING_THRESHOLD = 200 * 1000 * 1000

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.prefix = kwargs.get("prefix", "")
        self._destination = ""
        self.compression = kwargs.get("compression", "gz")
        self.compression_level = kwargs.get("compression_level", 6)
        self.interval = kwargs.get("interval", 1)
        self.time_interval = kwargs.get("time_interval", 15)
        self.time = 0
        self._skipped_counter = 0
        self.skip = Bool(False)
        self.warn_about_size = kwargs.get("warn_about_size", True)
        self.demand("suffix")

    @property
    def destination(self):
        return self._destination

    def initialize(self, **kwargs):
        self.time = time.time()

    def run(self):
        if get(root.common.disable.snapshotting, False) is True:
            return
        self._skipped_counter += 1
        if self._skipped_counter < self.interval or self.skip:
            return
        self._skipped_counter = 0
        # the run counter above is identical on every data-parallel rank;
        # the wall clocks are not, so the time gate is decided by rank 0 and
        # broadcast: every rank then enters (or skips) the barrier in
        # export_if_rank0 together (a rank skipping it while another waits
        # would pair the barrier with the next step's gradient all-reduce)
        due = time.time() - self.time >= self.time_interval
        dp = self._dp()
        if dp is not None and dp.world_size > 1:
            due = dp.agree(due)
        if not due:
            return
        self.export_if_rank0()
        return True

    def stop(self):
        if self._skipped_counter > 0 and not self.skip and \
                get(root.common.disable.snapshotting, False) is not True:
            self._skipped_counter = 0
            self.export_if_rank0()

    def _dp(self):
        from veles_amd.parallel import find_dp
        return find_dp(self)

    def export_if_rank0(self):
        dp = self._dp()
        if dp is not None and dp.world_size > 1:
            dp.barrier()
        if _rank() == 0:
            self.export()
        if dp is not None and dp.world_size > 1:
            # nobody starts the next interval before the file is complete,
            # and every rank restarts its interval clock at the same point
            dp.barrier()
        self.time = time.time()

    def export(self):
        raise NotImplementedError

    def check_snapshot_size(self, size):
        if size > self.SIZE_WARNING_THRESHOLD and self.warn_about_size:
            sizes = []
            for u in self.workflow:
                try:
                    sizes.append((len(pickle.dumps(u, PROTOCOL)), u.name))
                except Exception:
                    pass
            sizes.sort(reverse=True)
            self.warning("Snapshot size %.1f MB; biggest units: %s",
                         size / 1e6, ", ".join("%s %.1f MB" % (n, s / 1e6)
                                               for s, n in sizes[:5]))

    def get_metric_values(self):
        return {"Snapshot": self.destination}

    @staticmethod
    def import_(file_name):
        return import_snapshot(file_name)


class SnapshotterToFile(SnapshotterBase):
    MAPPING = "file"

    WRITE_CODECS = {
        None: lambda n, l: open(n, "wb"),
        "": lambda n, l: open(n, "wb"),
        "gz": lambda n, l: gzip.GzipFile(n, "wb", compresslevel=l),
        "bz2": lambda n, l: bz2.BZ2File(n, "wb", compresslevel=l),
        "xz": lambda n, l: lzma.LZMAFile(n, "wb", preset=l),
    }
    READ_CODECS = {
        "pickle": lambda n: open(n, "rb"),
        "gz": lambda n: gzip.GzipFile(n, "rb"),
        "bz2": lambda n: bz2.BZ2File(n, "rb"),
        "xz": lambda n: lzma.LZMAFile(n, "rb"),
    }

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.directory = kwargs.get("directory",
                                    get(root.common.dirs.snapshots, "."))
        # ensemble members / GA children share a config: keep their
        # snapshots apart
        idx = get(root.common.ensemble.model_index, None)
        if idx is not None:
            self.prefix = "%s_model%d" % (self.prefix, int(idx))
        if self.compression == "snappy":
            self.warning("snappy is unavailable; using gz")
            self.compression = "gz"

    def export(self):
        os.makedirs(self.directory, exist_ok=True)
        ext = ("." + self.compression) if self.compression else ""
        rel = "%s_%s.%d.pickle%s" % (self.prefix, self.suffix, PROTOCOL, ext)
        self._destination = os.path.abspath(os.path.join(self.directory, rel))
        self.info("Snapshotting to %s", self._destination)
        tmp = "%s.%d.tmp" % (self._destination, os.getpid())
        with self.WRITE_CODECS[self.compression](
                tmp, self.compression_level) as f:
            pickle.dump(self.workflow, f, protocol=PROTOCOL)
        os.replace(tmp, self._destination)
        self.check_snapshot_size(os.path.getsize(self._destination))
        link = os.path.join(self.directory, "%s_current.%d.pickle%s" % (
            self.prefix, PROTOCOL, ext))
        tmp_link = "%s.%d.tmp" % (link, os.getpid())
        try:
            os.symlink(rel, tmp_link)
            os.replace(tmp_link, link)  # atomic for concurrent writers
        except OSError:
            pass
        return self._destination

    @staticmethod
    def import_(file_name):
        """Load a snapshot written by this framework (own file: pickle)."""
        file_name = file_name.strip()
        if not os.path.exists(file_name):
            raise FileNotFoundError(file_name)
        ext = os.path.splitext(file_name)[1][1:]
        if ext == "snappy":
            raise ValueError("snappy snapshots are not supported")
        codec = SnapshotterToFile.READ_CODECS.get(
            ext, SnapshotterToFile.READ_CODECS["pickle"])
        logging.getLogger("Snapshotter").info("Reading %s", file_name)
        with codec(file_name) as f:
            return pickle.load(f)


class SnapshotterToDB(SnapshotterBase):
    """Snapshots into an SQLite table (id, prefix, suffix, timestamp,
    codec, data) - the reference's ODBC sink shape."""
    MAPPING = "db"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.database = kwargs.get("database", os.path.join(
            get(root.common.dirs.snapshots, "."), "snapshots.sqlite"))
        self.table = kwargs.get("table", "veles")

    def _conn(self):
        d = os.path.dirname(os.path.abspath(self.database))
        os.makedirs(d, exist_ok=True)
        c = sqlite3.connect(self.database)
        c.execute("CREATE TABLE IF NOT EXISTS %s (id INTEGER PRIMARY KEY, "
                  "prefix TEXT, suffix TEXT, timestamp REAL, codec TEXT, "
                  "data BLOB)" % self.table)
        return c

    def export(self):
        bio = io.BytesIO()
        with gzip.GzipFile(fileobj=bio, mode="wb",
                           compresslevel=self.compression_level) as f:
            pickle.dump(self.workflow, f, protocol=PROTOCOL)
        c = self._conn()
        with c:
            cur = c.execute("INSERT INTO %s (prefix, suffix, timestamp, codec,"
                            " data) VALUES (?, ?, ?, ?, ?)" % self.table,
                            (self.prefix, str(self.suffix), time.time(), "gz",
                             bio.getvalue()))
            rid = cur.lastrowid
        c.close()
        self._destination = "sqlite://%s/%s/%d" % (self.database, self.table,
                                                   rid)
        return self._destination

    @staticmethod
    def import_from(database, table="veles", row_id=None, spec=None):
        c = sqlite3.connect(database)
        if row_id is None:
            row = c.execute("SELECT id, data FROM %s ORDER BY id DESC LIMIT "
                            "1" % table).fetchone()
        else:
            row = c.execute("SELECT id, data FROM %s WHERE id=?" % table,
                            (row_id,)).fetchone()
        c.close()
        if row is None:
            raise LookupError("no snapshot row %s in %s table %s" % (
                "newest" if row_id is None else row_id, database, table))
        if spec is not None:
            import hashlib
            _record_loaded(spec, (len(row[1]), hashlib.sha1(
                row[1]).hexdigest(), "row %d" % row[0]))
        with gzip.GzipFile(fileobj=io.BytesIO(row[1])) as f:
            return pickle.load(f)


def _split_sqlite(spec):
    """sqlite://<database file>[/<table>[/<row id>]] (SnapshotterToDB's
    destination string) -> (database, table, row id or None)."""
    rest = spec[len("sqlite://"):]
    parts = rest.split("/")
    for i in range(len(parts), 0, -1):
        db = "/".join(parts[:i])
        if db and os.path.isfile(db):
            tail = [t for t in parts[i:] if t]
            if len(tail) > 2:
                break
            table = tail[0] if tail else "veles"
            rid = int(tail[1]) if len(tail) > 1 else None
            return db, table, rid
    raise FileNotFoundError("no SQLite snapshot database in %r" % spec)


def _fetch(url, directory=None):
    """Download an http(s) snapshot into the snapshot directory and return
    the local path.  The name keeps its codec extension; a file of that
    name already there is never overwritten (the reference's
    ``wget.download`` picks a new name too): the download gets a
    process-unique one instead.  The partial file is process-unique as
    well, so ranks of one node that fetch the same URL at once never write
    into each other's file."""
    import urllib.parse
    import urllib.request
    directory = directory or get(root.common.dirs.snapshots, ".")
    os.makedirs(directory, exist_ok=True)
    name = os.path.basename(urllib.parse.urlparse(url).path) or \
        "downloaded.pickle"
    dst = os.path.join(directory, name)
    n = 0
    while os.path.exists(dst):
        n += 1
        dst = os.path.join(directory, "dl%d-%d-%s" % (os.getpid(), n, name))
    tmp = "%s.%d.part" % (dst, os.getpid())
    try:
        with urllib.request.urlopen(url, timeout=60) as r, \
                open(tmp, "wb") as f:
            while True:
                chunk = r.read(1 << 20)
                if not chunk:
                    break
                f.write(chunk)
        os.replace(tmp, dst)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return dst


# spec -> (size, sha1, source) of the bytes import_snapshot actually loaded
_LOADED = {}


def _record_loaded(spec, digest):
    _LOADED[spec.strip()] = digest


def loaded_digest(spec):
    """(size, sha1 of the snapshot bytes, where they came from) that
    ``import_snapshot(spec)`` loaded in this process, or None.  For
    ``sqlite://`` and ``http(s)://`` specs the spec string alone does not
    say which bytes a rank restored (the newest row, a re-fetched URL):
    the launcher compares these digests across ranks instead."""
    return _LOADED.get(spec.strip())


def import_snapshot(spec):
    """``-w`` for every sink (reference veles/__main__.py:539-589): a file
    path, ``sqlite://db[/table[/id]]`` (SnapshotterToDB; newest row when
    the id is omitted) or an ``http(s)://`` URL (fetched into
    root.common.dirs.snapshots first).  What was loaded is recorded for
    ``loaded_digest``."""
    spec = spec.strip()
    if spec.startswith("sqlite://"):
        db, table, rid = _split_sqlite(spec)
        logging.getLogger("Snapshotter").info(
            "Reading %s table %s row %s", db, table,
            "newest" if rid is None else rid)
        return SnapshotterToDB.import_from(db, table, rid, spec=spec)
    if spec.startswith("odbc://"):
        raise ValueError("odbc:// snapshots: use the SQLite sink "
                         "(sqlite://<file>[/<table>[/<id>]])")
    path = _fetch(spec) if spec.startswith(("http://", "https://")) else spec
    from veles_amd.parallel.launch import snapshot_digest
    if os.path.isfile(path):
        _record_loaded(spec, snapshot_digest(path) + (path,))
    return SnapshotterToFile.import_(path)
