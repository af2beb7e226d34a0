"""Downloader: fetch a dataset archive into ``root.common.dirs.datasets`` and
unpack it (reference veles/downloader.py:56-125).

Differences from the reference: no ``wget`` dependency (``urllib`` handles
http(s) and ``file://``; a bare path is copied), archives are unpacked with
member-path checks so an archive cannot write outside ``directory``, and the
download is skipped when every required file is already readable - the
normal case on the GPU boxes, which have no network.
"""
from __future__ import annotations

import os
import shutil
import tarfile
import urllib.parse
import urllib.request
import zipfile

from veles_amd.distributable import TriviallyDistributable
from veles_amd.units import Unit
from veles_amd.utils.config import root, get

__all__ = ["Downloader", "fetch", "unpack"]


def fetch(url, directory):
    """Copy ``url`` (http(s)://, file:// or a local path) into
    ``directory``; returns the local file name."""
    parsed = urllib.parse.urlparse(url)
    name = os.path.basename(parsed.path) or "download"
    dst = os.path.join(directory, name)
    if parsed.scheme in ("", "file"):
        src = urllib.request.url2pathname(parsed.path) \
            if parsed.scheme == "file" else url
        shutil.copyfile(src, dst)
        return dst
    with urllib.request.urlopen(url) as r, open(dst, "wb") as f:
        shutil.copyfileobj(r, f, 1 << 20)
    return dst


def _safe_target(directory, member):
    target = os.path.realpath(os.path.join(directory, member))
    base = os.path.realpath(directory)
    if os.path.commonpath([target, base]) != base:
        raise ValueError("archive member %r escapes %s" % (member, directory))
    return target


def unpack(path, directory):
    """Extract a zip or tar(.gz/.bz2/.xz) archive; False if ``path`` is
    not an archive."""
    if zipfile.is_zipfile(path):
        with zipfile.ZipFile(path) as z:
            for m in z.namelist():
                _safe_target(directory, m)
            z.extractall(directory)
        return True
    if tarfile.is_tarfile(path):
        with tarfile.open(path) as t:
            members = t.getmembers()
            for m in members:
                _safe_target(directory, m.name)
                # a link member can be the first hop of a chain (d/l -> ..,
                # d/l/m -> .., d/l/m/x) that no per-member realpath check
                # sees before extraction: datasets need no links at all
                if m.issym() or m.islnk():
                    raise ValueError("archive member %r is a link" % m.name)
                if not (m.isfile() or m.isdir()):
                    raise ValueError("archive member %r is not a regular "
                                     "file or directory" % m.name)
            kw = {"filter": "data"} if hasattr(tarfile, "data_filter") else {}
            t.extractall(directory, members=members, **kw)
        return True
    return False


class Downloader(Unit, TriviallyDistributable):
    """``url``: what to fetch; ``files``: paths (relative to ``directory``)
    that must exist afterwards; ``directory``: defaults to
    ``root.common.dirs.datasets``."""

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.url = kwargs["url"]
        files = kwargs.get("files", ())
        self.files = {files} if isinstance(files, str) else set(files)
        self.directory = kwargs.get(
            "directory", get(root.common.dirs.datasets, "."))

    def _have_all(self):
        return bool(self.files) and all(
            os.access(os.path.join(self.directory, f), os.R_OK)
            for f in self.files)

    def initialize(self, **kwargs):
        if self._have_all():
            return
        os.makedirs(self.directory, exist_ok=True)
        if not os.access(self.directory, os.W_OK):
            raise PermissionError("cannot write to %s" % self.directory)
        self.info("Downloading %s to %s", self.url, self.directory)
        path = fetch(self.url, self.directory)
        if unpack(path, self.directory):
            os.remove(path)
        else:
            self.warning("%s is not a zip or tar archive; kept as is", path)
        missing = [f for f in self.files if not os.access(
            os.path.join(self.directory, f), os.R_OK)]
        if missing:
            raise FileNotFoundError("after downloading %s: missing %s" %
                                    (self.url, ", ".join(sorted(missing))))

    def run(self):
        pass
