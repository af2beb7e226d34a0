"""File scanning for the file-based loaders.

Reference: veles/loader/file_loader.py:48-297 — directory scan with MIME and
regex include / ignore filters, file lists, and the label derived from the
path (parent directory name or a regex group of the file name).
"""
from __future__ import annotations

import mimetypes
import os
import re

__all__ = ["FileFilter", "scan_files", "label_from_path", "read_file_list"]


class FileFilter(object):
    """``mime_types``: prefixes such as "image/"; ``filename_types``:
    extensions; ``included`` / ``ignored``: regexes on the full path."""

    def __init__(self, mime_types=("image/",), filename_types=None,
                 included=None, ignored=None):
        self.mime_types = tuple(mime_types or ())
        self.filename_types = tuple(
            e.lower().lstrip(".") for e in (filename_types or ()))
        self.included = [re.compile(r) for r in (included or ())]
        self.ignored = [re.compile(r) for r in (ignored or ())]

    def __call__(self, path):
        if any(r.search(path) for r in self.ignored):
            return False
        if self.included and not any(r.search(path) for r in self.included):
            return False
        ext = os.path.splitext(path)[1].lower().lstrip(".")
        if self.filename_types:
            return ext in self.filename_types
        if self.mime_types:
            mt = mimetypes.guess_type(path)[0] or ""
            return any(mt.startswith(m) for m in self.mime_types)
        return True


def scan_files(paths, file_filter=None):
    """Sorted list of files under ``paths`` (dirs scanned recursively)."""
    ff = file_filter or FileFilter()
    out = []
    for p in ([paths] if isinstance(paths, str) else paths):
        if os.path.isfile(p):
            if ff(p):
                out.append(p)
            continue
        for d, _, files in os.walk(p):
            for f in files:
                full = os.path.join(d, f)
                if ff(full):
                    out.append(full)
    return sorted(out)


def label_from_path(path, regexp=None):
    """The label of a file: a regex group of its base name, else the name of
    its directory (reference AutoLabelFileImageLoader)."""
    if regexp:
        m = re.search(regexp, os.path.basename(path))
        if m:
            return m.group(1) if m.groups() else m.group(0)
    return os.path.basename(os.path.dirname(path))


def read_file_list(path, base_dir=None):
    """Lines "file [label]" -> [(path, label or None)]."""
    base_dir = base_dir or os.path.dirname(os.path.abspath(path))
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            parts = line.split()
            fn = parts[0] if os.path.isabs(parts[0]) else os.path.join(
                base_dir, parts[0])
            out.append((fn, parts[1] if len(parts) > 1 else None))
    return out
