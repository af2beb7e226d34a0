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
