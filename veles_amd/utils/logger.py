"""Logging mixin and timeline events.

Reference: veles/logger.py:59-289 (``Logger`` mixin, ``ColorFormatter``,
``setup_logging``, ``redirect_all_logging_to_file``, ``event``).  The reference
records events into MongoDB; here events go to an in-memory buffer that is
flushed as Chrome-trace JSON (chrome://tracing / Perfetto) and/or JSONL, so
a rocprofv3 kernel trace and the unit timeline can be read side by side.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time

__all__ = ["Logger", "setup_logging", "redirect_all_logging_to_file",
           "EventRecorder", "events"]


class ColorFormatter(logging.Formatter):
    COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m",
              "ERROR": "\033[31m", "CRITICAL": "\033[1;31m"}
    RESET = "\033[0m"

    def __init__(self, color=True):
        super().__init__("%(asctime)s %(levelname)-7s %(name)s: %(message)s",
                         "%H:%M:%S")
        self.color = color

    def format(self, record):
        msg = super().format(record)
        if self.color:
            c = self.COLORS.get(record.levelname)
            if c:
                return c + msg + self.RESET
        return msg


_configured = False


def setup_logging(level=logging.INFO, color=None):
    global _configured
    if color is None:
        color = hasattr(sys.stderr, "isatty") and sys.stderr.isatty()
    rootlog = logging.getLogger()
    if not _configured:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(ColorFormatter(color))
        rootlog.addHandler(h)
        _configured = True
    rootlog.setLevel(level)


def redirect_all_logging_to_file(path, max_bytes=1 << 24, backups=3):
    from logging.handlers import RotatingFileHandler
    rootlog = logging.getLogger()
    for h in list(rootlog.handlers):
        rootlog.removeHandler(h)
    h = RotatingFileHandler(path, maxBytes=max_bytes, backupCount=backups)
    h.setFormatter(ColorFormatter(False))
    rootlog.addHandler(h)


class EventRecorder(object):
    """Collects begin/end/single events; dumps Chrome-trace JSON."""

    def __init__(self):
        self._lock = threading.Lock()
        self._events = []
        self.enabled = False
        self.pid = os.getpid()
        self.t0 = time.perf_counter()

    def record(self, name, kind, **info):
        if not self.enabled:
            return
        ph = {"begin": "B", "end": "E", "single": "i"}[kind]
        ev = {"name": name, "ph": ph, "pid": self.pid,
              "tid": threading.get_ident() & 0xFFFF,
              "ts": (time.perf_counter() - self.t0) * 1e6}
        if info:
            ev["args"] = {k: (v if isinstance(v, (int, float, str, bool))
                              else repr(v)) for k, v in info.items()}
        if ph == "i":
            ev["s"] = "t"
        with self._lock:
            self._events.append(ev)

    def complete(self, name, start_s, dur_s, **info):
        """Record a complete ("X") event, e.g. a HIP-event-timed unit run."""
        if not self.enabled:
            return
        ev = {"name": name, "ph": "X", "pid": self.pid,
              "tid": threading.get_ident() & 0xFFFF,
              "ts": (start_s - self.t0) * 1e6, "dur": dur_s * 1e6}
        if info:
            ev["args"] = info
        with self._lock:
            self._events.append(ev)

    @property
    def events(self):
        with self._lock:
            return list(self._events)

    def clear(self):
        with self._lock:
            self._events.clear()

    def dump(self, path):
        with self._lock:
            data = {"traceEvents": list(self._events),
                    "displayTimeUnit": "ms"}
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(data, f)
        return path


events = EventRecorder()


class Logger(object):
    """Per-class logger mixin (reference veles/logger.py:59-262)."""

    def __init__(self, **kwargs):
        self._logger_ = logging.getLogger(
            kwargs.get("logger_name", self.__class__.__name__))
        super().__init__()

    @property
    def logger(self):
        lg = getattr(self, "_logger_", None)
        if lg is None:
            lg = logging.getLogger(self.__class__.__name__)
            self._logger_ = lg
        return lg

    def init_unpickled(self):
        sup = super()
        if hasattr(sup, "init_unpickled"):
            sup.init_unpickled()
        self._logger_ = logging.getLogger(self.__class__.__name__)

    def debug(self, msg, *args, **kw):
        self.logger.debug(msg, *args, **kw)

    def info(self, msg, *args, **kw):
        self.logger.info(msg, *args, **kw)

    def warning(self, msg, *args, **kw):
        self.logger.warning(msg, *args, **kw)

    def error(self, msg, *args, **kw):
        self.logger.error(msg, *args, **kw)

    def exception(self, msg="Exception", *args, **kw):
        self.logger.exception(msg, *args, **kw)

    def critical(self, msg, *args, **kw):
        self.logger.critical(msg, *args, **kw)

    def event(self, name, etype, **info):
        """Timeline event: etype in {"begin", "end", "single"}."""
        events.record(name, etype, cls=self.__class__.__name__, **info)
