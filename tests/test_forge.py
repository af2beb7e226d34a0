"""Forge package registry (reference veles/forge/*): upload
with tokens and ownership, HEAD / HEAD@{n} / explicit versions, list,
details, fetch + unpack, delete."""
import json
import urllib.error

import pytest

from veles_amd.forge import ForgeClient, ForgeServer


def _pkg(d, version, text):
    d.mkdir(exist_ok=True)
    (d / "manifest.json").write_text(json.dumps({
        "name": "mnist_fc", "workflow": "mnist_fc.py",
        "configuration": "mnist_fc_config.py", "short_description": "MLP",
        "author": "tester", "version": version, "requires": []}))
    (d / "mnist_fc.py").write_text(text)
    (d / "mnist_fc_config.py").write_text("root.x = 1\n")


def test_forge_roundtrip(tmp_path):
    srv = ForgeServer(str(tmp_path / "store"), tokens=["alice", "bob"])
    srv.start()
    try:
        c = ForgeClient(srv.url)
        src = tmp_path / "pkg"
        _pkg(src, "1.0", "v1\n")
        assert c.upload(str(src), "alice") == "OK"
        _pkg(src, "1.1", "v2\n")
        c.upload(str(src), "alice")
        lst = c.list()
        assert [p["name"] for p in lst] == ["mnist_fc"]
        assert lst[0]["version"] == "1.1"
        det = c.details("mnist_fc")
        assert [v["version"] for v in det["versions"]] == ["1.0", "1.1"]
        assert "owner" not in det
        c.fetch("mnist_fc", str(tmp_path / "head"))
        assert (tmp_path / "head" / "mnist_fc.py").read_text() == "v2\n"
        c.fetch("mnist_fc", str(tmp_path / "prev"), version="HEAD@{1}")
        assert (tmp_path / "prev" / "mnist_fc.py").read_text() == "v1\n"
        c.fetch("mnist_fc", str(tmp_path / "v10"), version="1.0")
        assert (tmp_path / "v10" / "mnist_fc.py").read_text() == "v1\n"
        # unknown token, other owner, duplicate version
        for tok, ver in (("mallory", "2.0"), ("bob", "2.0"),
                         ("alice", "1.1")):
            _pkg(src, ver, "x\n")
            with pytest.raises(urllib.error.HTTPError) as e:
                c.upload(str(src), tok)
            assert e.value.code in (400, 403)
        with pytest.raises(urllib.error.HTTPError) as e:
            c.delete("mnist_fc", "bob")
        assert e.value.code == 403
        assert c.delete("mnist_fc", "alice") == "OK"
        assert c.list() == []
        with pytest.raises(urllib.error.HTTPError) as e:
            c.details("mnist_fc")
        assert e.value.code == 404
    finally:
        srv.stop()


@pytest.mark.parametrize("bad", [".", "..", ".hidden", "", "a/b", "../x"])
def test_forge_rejects_dot_names(tmp_path, bad):
    """'..' used to resolve to the store's parent: an upload wrote there and
    a delete removed the whole store."""
    from veles_amd.forge import ForgeStore
    root = tmp_path / "store"
    st = ForgeStore(str(root), tokens=["alice"])
    (tmp_path / "keep.txt").write_text("k")
    meta = {"name": bad, "workflow": "w.py", "configuration": "c.py",
            "short_description": "d", "author": "a", "version": "1"}
    import io
    import tarfile
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as t:
        ti = tarfile.TarInfo("w.py")
        ti.size = 0
        t.addfile(ti, io.BytesIO(b""))
    with pytest.raises(KeyError):
        st.upload("alice", meta, buf.getvalue())
    with pytest.raises(KeyError):
        st.delete("alice", bad)
    assert (tmp_path / "keep.txt").exists()
    assert (root / "tokens.json").exists()
    assert not (tmp_path / "manifest.json").exists()


def test_forge_http_delete_dotdot(tmp_path):
    srv = ForgeServer(str(tmp_path / "store"), tokens=["alice"])
    srv.start()
    try:
        c = ForgeClient(srv.url)
        with pytest.raises(urllib.error.HTTPError) as e:
            c.delete("..", "alice")
        assert e.value.code in (400, 403, 404)
        assert (tmp_path / "store" / "tokens.json").exists()
    finally:
        srv.stop()
