"""``-w`` restores from every snapshot sink (reference veles/__main__.py:
539-589 accepts files, ``odbc://`` and ``http(s)://``): a file, the SQLite
sink's ``sqlite://db/table/id`` destination (newest row without an id) and
an ``http://`` URL fetched into the snapshot directory - through
``snapshotter.import_snapshot`` and through the CLI."""
import functools
import http.server
import os
import sys
import threading

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MOD = '''
from veles_amd.units import TrivialUnit
from veles_amd.workflow import Workflow


class Count(TrivialUnit):
    def __init__(self, workflow, **kw):
        super().__init__(workflow, **kw)
        self.n = 0

    def run(self):
        self.n += 1


class CountWF(Workflow):
    def __init__(self, launcher, **kw):
        super().__init__(launcher, **kw)
        self.count = Count(self)
        self.count.link_from(self.start_point)
        self.end_point.link_from(self.count)
'''

WF = '''
from snapwf_mod import CountWF

def run(load, main):
    load(CountWF)
    main()
'''


@pytest.fixture
def snapmod(tmp_path, monkeypatch):
    (tmp_path / "snapwf_mod.py").write_text(MOD)
    monkeypatch.syspath_prepend(str(tmp_path))
    sys.modules.pop("snapwf_mod", None)
    import snapwf_mod
    return snapwf_mod


def _wf(mod, n):
    from veles_amd.dummy import DummyLauncher
    wf = mod.CountWF(DummyLauncher())
    wf.count.n = n
    return wf


def test_sqlite_newest_and_by_id(snapmod, tmp_path):
    from veles_amd.snapshotter import SnapshotterToDB, import_snapshot
    db = str(tmp_path / "snaps" / "s.sqlite")
    dests = []
    for n in (3, 7):
        wf = _wf(snapmod, n)
        s = SnapshotterToDB(wf, database=db, prefix="cnt")
        dests.append(s.export())
    assert dests[0].startswith("sqlite://" + db + "/veles/")
    assert import_snapshot(dests[0]).count.n == 3
    assert import_snapshot(dests[1]).count.n == 7
    # no row id: the newest row; no table either: the default table
    assert import_snapshot("sqlite://%s/veles" % db).count.n == 7
    assert import_snapshot("sqlite://%s" % db).count.n == 7
    with pytest.raises(FileNotFoundError):
        import_snapshot("sqlite://%s/none.sqlite/veles/1" % tmp_path)


def test_http_snapshot_fetched(snapmod, tmp_path):
    from veles_amd.snapshotter import SnapshotterToFile, import_snapshot
    from veles_amd.utils.config import root
    src = tmp_path / "srv"
    src.mkdir()
    wf = _wf(snapmod, 11)
    s = SnapshotterToFile(wf, directory=str(src), prefix="cnt",
                          compression="gz")
    path = s.export()
    handler = functools.partial(http.server.SimpleHTTPRequestHandler,
                                directory=str(src))
    httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    t = threading.Thread(target=httpd.serve_forever, daemon=True)
    t.start()
    old = root.common.dirs.snapshots
    root.common.dirs.snapshots = str(tmp_path / "dl")
    try:
        url = "http://127.0.0.1:%d/%s" % (httpd.server_address[1],
                                          os.path.basename(path))
        wf2 = import_snapshot(url)
        assert wf2.count.n == 11
        assert os.path.isfile(tmp_path / "dl" / os.path.basename(path))
    finally:
        root.common.dirs.snapshots = old
        httpd.shutdown()


def test_loaded_digest_names_the_restored_row(snapmod, tmp_path):
    """the multi-rank "same snapshot" check digests the bytes a
    rank restored, not the spec string - a sqlite:// spec without a row id
    names whatever row is newest when the rank reads it."""
    from veles_amd.snapshotter import (SnapshotterToDB, import_snapshot,
                                       loaded_digest)
    db = str(tmp_path / "d.sqlite")
    SnapshotterToDB(_wf(snapmod, 1), database=db, prefix="c").export()
    spec = "sqlite://%s" % db
    assert import_snapshot(spec).count.n == 1
    first = loaded_digest(spec)
    assert first[2] == "row 1"
    SnapshotterToDB(_wf(snapmod, 2), database=db, prefix="c").export()
    assert import_snapshot(spec).count.n == 2
    second = loaded_digest(spec)
    assert second[2] == "row 2" and second[:2] != first[:2]


def test_http_fetch_never_overwrites_and_is_unique(snapmod, tmp_path):
    """a local file with the URL's basename is kept, and the
    download lands under a new name."""
    from veles_amd.snapshotter import (SnapshotterToFile, _fetch,
                                       loaded_digest, import_snapshot)
    src = tmp_path / "srv"
    src.mkdir()
    path = SnapshotterToFile(_wf(snapmod, 4), directory=str(src),
                             prefix="cnt", compression="gz").export()
    handler = functools.partial(http.server.SimpleHTTPRequestHandler,
                                directory=str(src))
    httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    t = threading.Thread(target=httpd.serve_forever, daemon=True)
    t.start()
    try:
        dl = tmp_path / "dl"
        dl.mkdir()
        keep = dl / os.path.basename(path)
        keep.write_bytes(b"local file")
        url = "http://127.0.0.1:%d/%s" % (httpd.server_address[1],
                                          os.path.basename(path))
        got = _fetch(url, str(dl))
        assert keep.read_bytes() == b"local file"
        assert got != str(keep) and got.endswith(".gz")
        got2 = _fetch(url, str(dl))
        assert got2 not in (got, str(keep))
        assert not [f for f in os.listdir(dl) if f.endswith(".part")]
        from veles_amd.utils.config import root
        old = root.common.dirs.snapshots
        root.common.dirs.snapshots = str(dl)
        try:
            assert import_snapshot(url).count.n == 4
        finally:
            root.common.dirs.snapshots = old
        d = loaded_digest(url)
        assert d is not None and d[0] == os.path.getsize(path)
    finally:
        httpd.shutdown()


def test_cli_resumes_from_sqlite(snapmod, tmp_path):
    from veles_amd.__main__ import Main
    from veles_amd.snapshotter import SnapshotterToDB
    db = str(tmp_path / "s.sqlite")
    snap = SnapshotterToDB(_wf(snapmod, 5), database=db, prefix="cnt")
    snap.suffix = "t"   # a snapshotter unit rides along in the snapshot
    dest = snap.export()
    p = tmp_path / "snapwf.py"
    p.write_text(WF)
    m = Main([str(p), "", "-a", "cpu", "-w", dest])
    assert m.run() == 0
    # restored at n = 5, then one pass of the workflow
    assert m.workflow.count.n == 6
