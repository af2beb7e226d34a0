"""Run status reporting (reference veles/web_status.py:113-314 and the
launcher's status POSTs, launcher.py:852-885).

The reference pushes a JSON status to a Tornado dashboard every
``notification_interval`` seconds.  Here ``StatusReporter`` appends the same
kind of record (workflow, epoch, metrics, per-unit timings, device memory,
rank) to a JSONL file and optionally serves the latest records over HTTP
(``GET /status``, stdlib server) — no Mongo, no Tornado.
"""
from __future__ import annotations

import json
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from veles_amd.units import Unit
from veles_amd.utils.json_encoders import NumpyJSONEncoder

__all__ = ["StatusReporter", "collect_status", "prometheus_text"]


def prometheus_text(st, prefix="veles_amd"):
    """Prometheus text exposition (format 0.0.4) of one status record:
    numeric scalars become gauges, per-unit run times one labelled gauge,
    and every sample carries the rank label (a scrape target per rank)."""
    import re
    rank = st.get("rank", 0)
    lines = []

    def gauge(name, value, labels=""):
        name = prefix + "_" + re.sub(r"[^a-zA-Z0-9_]", "_", name)
        lab = 'rank="%s"%s' % (rank, labels)
        lines.append("# TYPE %s gauge" % name)
        lines.append("%s{%s} %r" % (name, lab, float(value)))

    def walk(key, v):
        if isinstance(v, bool):
            gauge(key, int(v))
        elif isinstance(v, (int, float)):
            gauge(key, v)
        elif isinstance(v, dict) and key != "units":
            for k, x in v.items():
                walk(key + "_" + str(k), x)
    for k, v in st.items():
        if k not in ("rank", "pid"):
            walk(k, v)
    units = st.get("units") or {}
    if units:
        name = prefix + "_unit_run_seconds"
        lines.append("# TYPE %s gauge" % name)
        for u, t in units.items():
            lines.append('%s{rank="%s",unit="%s"} %r' % (
                name, rank, str(u).replace("\\", "_").replace('"', "'"),
                float(t)))
    return "\n".join(lines) + "\n"


def collect_status(wf):
    st = {"time": time.time(), "workflow": getattr(wf, "name", ""),
          "class": type(wf).__name__, "pid": os.getpid(),
          "rank": int(os.environ.get("RANK", "0"))}
    d = getattr(wf, "decision", None)
    if d is not None:
        st["epoch"] = getattr(d, "epoch_number", None)
        hist = getattr(d, "history", None)
        if hist:
            st["last_epoch"] = hist[-1]
    ld = getattr(wf, "loader", None)
    if ld is not None:
        st["samples_served"] = getattr(ld, "samples_served", None)
    st["units"] = {u.name: round(getattr(u, "total_run_time", 0.0), 6)
                   for u in wf if u is not wf}
    try:
        import torch
        if torch.cuda.is_available():
            st["device_memory"] = {
                "allocated": torch.cuda.memory_allocated(),
                "peak": torch.cuda.max_memory_allocated()}
    except Exception:
        pass
    return st


class StatusReporter(Unit):
    MAPPING = "status_reporter"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.file = kwargs.get("file", "status.jsonl")
        self.interval = float(kwargs.get("notification_interval", 1.0))
        self.port = kwargs.get("port")
        self.keep = int(kwargs.get("keep", 100))
        self.records = []
        self.last = 0.0

    def init_unpickled(self):
        super().init_unpickled()
        self.server_ = None

    def initialize(self, **kwargs):
        if self.port is None or self.server_ is not None:
            return
        rep = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path.rstrip("/") == "/metrics":
                    st = rep.records[-1] if rep.records else {}
                    body = prometheus_text(st).encode()
                    self.send_response(200)
                    self.send_header("Content-Type",
                                     "text/plain; version=0.0.4")
                    self.end_headers()
                    self.wfile.write(body)
                    return
                if self.path.rstrip("/") not in ("/status", ""):
                    self.send_response(404)
                    self.end_headers()
                    return
                body = json.dumps(rep.records[-1:] and rep.records[-1],
                                  cls=NumpyJSONEncoder).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.end_headers()
                self.wfile.write(body)

        self.server_ = ThreadingHTTPServer(("127.0.0.1", int(self.port)), H)
        self.port = self.server_.server_address[1]
        threading.Thread(target=self.server_.serve_forever,
                         daemon=True).start()

    def run(self):
        now = time.time()
        if now - self.last < self.interval:
            return
        self.last = now
        self.report()

    def report(self):
        st = collect_status(self.workflow)
        self.records.append(st)
        del self.records[:-self.keep]
        with open(self.file, "a") as f:
            f.write(json.dumps(st, cls=NumpyJSONEncoder) + "\n")
        return st

    def stop(self):
        self.report()
        if self.server_ is not None:
            self.server_.shutdown()
            self.server_.server_close()
            self.server_ = None
