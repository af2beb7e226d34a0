"""RESTful inference API (reference veles/restful_api.py:54-217).

Clients POST JSON ``{"input": [...] | "<base64>", "codec": "list" |
"base64", "shape": [...], "type": "float32"}`` to ``/service``; the sample
is fed to a ``RestfulLoader``; after the forward pass this unit answers
every request of the minibatch with ``{"result": <output row>,
"label": <argmax label>}``.  Standard-library HTTP server in a daemon
thread (no Twisted); the forward pass runs on the MI355X through the
ordinary workflow, several queued requests batched into one minibatch.
"""
from __future__ import annotations

import base64
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy

from veles_amd.units import Unit

__all__ = ["RESTfulAPI", "Request"]


class Request(object):
    __slots__ = ("event", "result", "error")

    def __init__(self):
        self.event = threading.Event()
        self.result = None
        self.error = None


def decode_input(msg):
    codec = msg.get("codec", "list")
    dt = numpy.dtype(msg.get("type", "float32"))
    if codec == "list":
        a = numpy.asarray(msg["input"], dtype=dt)
    elif codec == "base64":
        a = numpy.frombuffer(base64.b64decode(msg["input"]), dtype=dt)
    else:
        raise ValueError("unknown codec %r" % codec)
    if "shape" in msg:
        a = a.reshape(msg["shape"])
    return a


class RESTfulAPI(Unit):
    MAPPING = "restful_api"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.host = kwargs.get("host", "127.0.0.1")
        self.port = int(kwargs.get("port", 0))
        self.path = kwargs.get("path", "/service")
        self.timeout = float(kwargs.get("timeout", 60.0))
        self.loader = kwargs.get("loader")
        self.demand("output")

    def init_unpickled(self):
        super().init_unpickled()
        self.server_ = None
        self.thread_ = None

    def initialize(self, **kwargs):
        if self.loader is None:
            self.loader = getattr(self.workflow, "loader", None)
        if self.server_ is not None:
            return
        api = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *args):
                pass

            def _reply(self, code, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                if self.path != api.path:
                    return self._reply(404, {"error": "not found"})
                try:
                    n = int(self.headers.get("Content-Length", "0"))
                    msg = json.loads(self.rfile.read(n))
                    x = decode_input(msg)
                except Exception as e:
                    return self._reply(400, {"error": str(e)})
                req = Request()
                api.loader.feed(x, req)
                if not req.event.wait(api.timeout):
                    return self._reply(504, {"error": "timeout"})
                if req.error:
                    return self._reply(500, {"error": req.error})
                return self._reply(200, req.result)

        self.server_ = ThreadingHTTPServer((self.host, self.port), Handler)
        self.port = self.server_.server_address[1]
        self.thread_ = threading.Thread(target=self.server_.serve_forever,
                                        daemon=True)
        self.thread_.start()
        self.info("RESTful API on http://%s:%d%s", self.host, self.port,
                  self.path)

    def run(self):
        reqs = getattr(self.loader, "current_requests", [])
        if not reqs:
            return
        out = self.output.devmem
        rows = out[:len(reqs)].float().reshape(len(reqs), -1).cpu().numpy()
        labels = getattr(self.loader, "reversed_labels_mapping", None)
        for row, req in zip(rows, reqs):
            if req is None:
                continue
            res = {"result": row.tolist()}
            k = int(row.argmax())
            res["label"] = labels[k] if labels and k < len(labels) else k
            req.result = res
            req.event.set()

    def stop(self):
        if self.server_ is not None:
            self.server_.shutdown()
            self.server_.server_close()
            self.server_ = None
