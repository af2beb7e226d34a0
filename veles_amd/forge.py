"""Forge: a registry of workflow packages (reference veles/forge/
forge_server.py:80-915, forge_client.py:91-799).

The reference keeps one git repository per package behind a Tornado server
with e-mail registration.  Here a package is a versioned directory of
``.tar.gz`` snapshots with a ``manifest.json``, served by a stdlib
``ThreadingHTTPServer`` - no git, Tornado or SMTP on the GPU boxes.

Kept from the reference:

* service queries ``list`` / ``details`` / ``delete`` (``GET
  /service?query=...``), ``GET /fetch?name=&version=`` returning a tar.gz,
  ``POST /upload?token=`` carrying the metadata JSON and the archive;
* version references ``HEAD`` (newest), ``HEAD@{n}`` (n uploads back) or an
  explicit version string;
* write access by token: only a known token may upload, and only the
  package's owner token may delete or upload a new version of it; tokens are
  stored scrambled (SHA-256);
* the manifest must name ``name``, ``workflow``, ``configuration``,
  ``short_description``, ``author`` and ``version``.

Client: ``ForgeClient(url).upload(path, token)``, ``.fetch(name, dest)``,
``.list()``, ``.details(name)``, ``.delete(name, token)``; CLI:
``python -m veles_amd.forge {serve,list,details,fetch,upload,delete}``.
"""
from __future__ import annotations

import argparse
import hashlib
import io
import json
import os
import re
import shutil
import struct
import tarfile
import threading
import time
import urllib.parse
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

__all__ = ["ForgeStore", "ForgeServer", "ForgeClient", "REQUIRED_FIELDS"]

REQUIRED_FIELDS = ("name", "workflow", "configuration", "short_description",
                   "author", "version")
# a name is one path component: it may not be empty, start with '.', or be
# '.' / '..' (which would put the package at or above the store root)
_NAME = re.compile(r"^[A-Za-z0-9_][A-Za-z0-9_.-]*$")


def scramble(token):
    return hashlib.sha256(token.encode()).hexdigest()


def _safe_extract(tar, dest):
    base = os.path.realpath(dest)
    for m in tar.getmembers():
        target = os.path.realpath(os.path.join(dest, m.name))
        if os.path.commonpath([target, base]) != base or m.issym() or \
                m.islnk():
            raise ValueError("unsafe archive member %r" % m.name)
    tar.extractall(dest)


class ForgeStore(object):
    """On-disk registry: ``root/<name>/manifest.json`` + ``<n>.tar.gz``."""

    def __init__(self, root, tokens=()):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self._lock = threading.Lock()
        self.tokens_file = os.path.join(root, "tokens.json")
        known = set()
        if os.path.exists(self.tokens_file):
            with open(self.tokens_file) as f:
                known = set(json.load(f))
        known.update(scramble(t) for t in tokens)
        self.tokens = known
        self._save_tokens()

    def _save_tokens(self):
        with open(self.tokens_file, "w") as f:
            json.dump(sorted(self.tokens), f)

    def add_token(self, token):
        with self._lock:
            self.tokens.add(scramble(token))
            self._save_tokens()

    def _dir(self, name):
        if not _NAME.match(name or ""):
            raise KeyError("bad package name %r" % name)
        path = os.path.join(self.root, name)
        # belt and braces: the package directory must be a direct child of
        # the store root even if the root itself is reached via symlinks
        if os.path.dirname(os.path.realpath(path)) != \
                os.path.realpath(self.root):
            raise KeyError("bad package name %r" % name)
        return path

    def _manifest(self, name):
        p = os.path.join(self._dir(name), "manifest.json")
        if not os.path.exists(p):
            raise KeyError(name)
        with open(p) as f:
            return json.load(f)

    def list(self):
        out = []
        for name in sorted(os.listdir(self.root)):
            if os.path.isdir(os.path.join(self.root, name)):
                m = self._manifest(name)
                out.append({"name": name, "description":
                            m["short_description"], "author": m["author"],
                            "version": m["versions"][-1]["version"],
                            "uploaded": m["versions"][-1]["time"]})
        return out

    def details(self, name):
        m = dict(self._manifest(name))
        m.pop("owner", None)
        return m

    def resolve(self, name, version="HEAD"):
        vs = self._manifest(name)["versions"]
        rel = re.match(r"^HEAD(?:@\{(\d+)\})?$", version or "HEAD")
        if rel:
            back = int(rel.group(1) or 0)
            if back >= len(vs):
                raise KeyError("%s has %d versions" % (name, len(vs)))
            return vs[-1 - back]
        for v in reversed(vs):
            if v["version"] == version:
                return v
        raise KeyError("%s: no version %s" % (name, version))

    def fetch(self, name, version="HEAD"):
        v = self.resolve(name, version)
        with open(os.path.join(self._dir(name), v["file"]), "rb") as f:
            return f.read()

    def upload(self, token, metadata, archive):
        if scramble(token) not in self.tokens:
            raise PermissionError("token is not allowed to write")
        missing = [k for k in REQUIRED_FIELDS if k not in metadata]
        if missing:
            raise ValueError("metadata lacks %s" % ", ".join(missing))
        tarfile.open(fileobj=io.BytesIO(archive), mode="r:gz").getmembers()
        name = metadata["name"]
        d = self._dir(name)
        with self._lock:
            os.makedirs(d, exist_ok=True)
            mp = os.path.join(d, "manifest.json")
            if os.path.exists(mp):
                m = self._manifest(name)
                if m["owner"] != scramble(token):
                    raise PermissionError("%s belongs to another token" %
                                          name)
            else:
                m = {"owner": scramble(token), "versions": []}
            if any(v["version"] == metadata["version"]
                   for v in m["versions"]):
                raise ValueError("%s %s already exists" %
                                 (name, metadata["version"]))
            fn = "%d.tar.gz" % len(m["versions"])
            with open(os.path.join(d, fn), "wb") as f:
                f.write(archive)
            m.update({k: v for k, v in metadata.items() if k != "owner"})
            m["versions"].append({"version": metadata["version"],
                                  "file": fn, "time": time.time()})
            with open(mp + ".tmp", "w") as f:
                json.dump(m, f, indent=1)
            os.replace(mp + ".tmp", mp)

    def delete(self, token, name):
        with self._lock:
            if self._manifest(name)["owner"] != scramble(token):
                raise PermissionError("only the owner may delete %s" % name)
            shutil.rmtree(self._dir(name))


class _Handler(BaseHTTPRequestHandler):
    store = None

    def log_message(self, fmt, *args):
        pass

    def _reply(self, code, body, ctype="application/json"):
        if isinstance(body, (dict, list)):
            body = json.dumps(body).encode()
        elif isinstance(body, str):
            body = body.encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _args(self):
        u = urllib.parse.urlparse(self.path)
        return u.path, {k: v[-1] for k, v in
                        urllib.parse.parse_qs(u.query).items()}

    def _guard(self, fn):
        try:
            return fn()
        except PermissionError as e:
            self._reply(403, {"error": str(e)})
        except KeyError as e:
            self._reply(404, {"error": str(e)})
        except (ValueError, tarfile.TarError) as e:
            self._reply(400, {"error": str(e)})

    def do_GET(self):
        path, a = self._args()
        st = self.store
        if path == "/service":
            q = a.get("query")
            if q == "list":
                return self._guard(lambda: self._reply(200, st.list()))
            if q == "details":
                return self._guard(lambda: self._reply(
                    200, st.details(a.get("name"))))
            if q == "delete":
                def go():
                    st.delete(a.get("token", ""), a.get("name"))
                    self._reply(200, "OK", "text/plain")
                return self._guard(go)
            return self._reply(400, {"error": "unknown query %r" % q})
        if path == "/fetch":
            return self._guard(lambda: self._reply(
                200, st.fetch(a.get("name"), a.get("version", "HEAD")),
                "application/x-gzip"))
        self._reply(404, {"error": "no such endpoint"})

    def do_POST(self):
        path, a = self._args()
        if path != "/upload":
            return self._reply(404, {"error": "no such endpoint"})
        n = int(self.headers.get("Content-Length", 0))
        body = self.rfile.read(n)

        def go():
            (ml,) = struct.unpack("<I", body[:4])
            meta = json.loads(body[4:4 + ml].decode())
            self.store.upload(a.get("token", ""), meta, body[4 + ml:])
            self._reply(200, "OK", "text/plain")
        self._guard(go)


class ForgeServer(object):
    def __init__(self, root, host="127.0.0.1", port=0, tokens=()):
        self.store = ForgeStore(root, tokens)
        handler = type("Handler", (_Handler,), {"store": self.store})
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.port = self.httpd.server_address[1]
        self.url = "http://%s:%d" % (host, self.port)
        self._thread = None

    def start(self):
        self._thread = threading.Thread(target=self.httpd.serve_forever,
                                        daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


class ForgeClient(object):
    def __init__(self, url):
        self.url = url.rstrip("/")

    def _get(self, path, **q):
        with urllib.request.urlopen("%s%s?%s" % (
                self.url, path, urllib.parse.urlencode(q))) as r:
            return r.read()

    def list(self):
        return json.loads(self._get("/service", query="list"))

    def details(self, name):
        return json.loads(self._get("/service", query="details", name=name))

    def delete(self, name, token):
        return self._get("/service", query="delete", name=name,
                         token=token).decode()

    def fetch(self, name, dest, version="HEAD"):
        """Download and unpack ``name`` into ``dest``; returns its
        manifest (``manifest.json`` inside the package)."""
        data = self._get("/fetch", name=name, version=version)
        os.makedirs(dest, exist_ok=True)
        with tarfile.open(fileobj=io.BytesIO(data), mode="r:gz") as t:
            _safe_extract(t, dest)
        mp = os.path.join(dest, "manifest.json")
        if os.path.exists(mp):
            with open(mp) as f:
                return json.load(f)
        return {}

    def upload(self, path, token, version=None):
        """Upload the package directory ``path`` (its ``manifest.json``
        supplies the metadata; ``version`` overrides)."""
        with open(os.path.join(path, "manifest.json")) as f:
            meta = json.load(f)
        if version is not None:
            meta["version"] = version
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:gz") as t:
            for f in sorted(os.listdir(path)):
                t.add(os.path.join(path, f), arcname=f)
        m = json.dumps(meta).encode()
        body = struct.pack("<I", len(m)) + m + buf.getvalue()
        req = urllib.request.Request(
            "%s/upload?%s" % (self.url, urllib.parse.urlencode(
                {"token": token})), data=body, method="POST")
        with urllib.request.urlopen(req) as r:
            return r.read().decode()


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m veles_amd.forge")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve")
    s.add_argument("-r", "--root", required=True)
    s.add_argument("-p", "--port", type=int, default=8090)
    s.add_argument("--host", default="127.0.0.1")
    s.add_argument("--token", action="append", default=[])
    for c in ("list", "details", "fetch", "upload", "delete"):
        p = sub.add_parser(c)
        p.add_argument("-s", "--server", default="http://127.0.0.1:8090")
        if c in ("details", "fetch", "delete"):
            p.add_argument("name")
        if c == "fetch":
            p.add_argument("-d", "--dest", default=".")
            p.add_argument("--version", default="HEAD")
        if c == "upload":
            p.add_argument("path")
            p.add_argument("--version", default=None)
        if c in ("upload", "delete"):
            p.add_argument("-t", "--token", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "serve":
        srv = ForgeServer(a.root, a.host, a.port, a.token)
        print("forge serving %s at %s" % (a.root, srv.url), flush=True)
        srv.httpd.serve_forever()
        return 0
    c = ForgeClient(a.server)
    if a.cmd == "list":
        out = c.list()
    elif a.cmd == "details":
        out = c.details(a.name)
    elif a.cmd == "fetch":
        out = c.fetch(a.name, a.dest, a.version)
    elif a.cmd == "upload":
        out = c.upload(a.path, a.token, a.version)
    else:
        out = c.delete(a.name, a.token)
    print(json.dumps(out, indent=1) if not isinstance(out, str) else out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
