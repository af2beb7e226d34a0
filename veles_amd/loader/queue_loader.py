"""Socket request queue feeding a workflow - the ZeroMQ loader's role
(reference veles/zmq_loader.py:74-138, ``ZeroMQLoader``) without ZeroMQ or
Twisted.

A listener thread accepts TCP (127.0.0.1 by default) or UNIX-socket
connections.  Each request frame is ``u32 length + .npy bytes``; it is queued
with its connection id.  ``run()`` first answers the previous request
(``reply_fn(workflow)``, default ``workflow.generate_data_for_master()``,
sent as a length-prefixed JSON frame) and then blocks for the next request,
which becomes ``output``.  ``stop()`` unblocks ``run()`` with ``None``.
The bound endpoints are reported to the master through
``generate_data_for_master`` exactly like the reference's
``ZmqLoaderEndpoints``.
"""
from __future__ import annotations

import io
import json
import os
import queue
import socket
import struct
import tempfile
import threading

import numpy

from veles_amd.distributable import IDistributable
from veles_amd.units import Unit
from veles_amd.utils.json_encoders import NumpyJSONEncoder

__all__ = ["QueueLoader", "QueueLoaderClient", "send_frame", "recv_frame"]


def send_frame(sock, payload):
    sock.sendall(struct.pack("<I", len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            return None
        buf += chunk
    return bytes(buf)


def recv_frame(sock):
    hdr = _recv_exact(sock, 4)
    if hdr is None:
        return None
    return _recv_exact(sock, struct.unpack("<I", hdr)[0])


class QueueLoader(Unit, IDistributable):
    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "LOADER")
        super().__init__(workflow, **kwargs)
        self.queue_size = int(kwargs.get("queue_size", 0))
        self.transport = kwargs.get("transport", "tcp")  # or "ipc"
        self.host = kwargs.get("host", "127.0.0.1")
        self.reply_fn = kwargs.get("reply_fn")
        self.output = None
        self.cid = None
        self.endpoints = {}

    def init_unpickled(self):
        super().init_unpickled()
        self._queue_ = queue.Queue(getattr(self, "queue_size", 0))
        self._conns_ = {}
        self._server_ = None
        self._threads_ = []

    # ---------------------------------------------------------- transport
    def initialize(self, **kwargs):
        if self.transport == "ipc":
            path = os.path.join(tempfile.mkdtemp(prefix="veles-ql-"), "sock")
            srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            srv.bind(path)
            self.endpoints = {"ipc": path}
        else:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((self.host, 0))
            self.endpoints = {"tcp": "%s:%d" % srv.getsockname()}
        srv.listen(16)
        self._server_ = srv
        t = threading.Thread(target=self._accept, daemon=True,
                             name="%s-accept" % self.name)
        t.start()
        self._threads_.append(t)

    def _accept(self):
        n = 0
        while True:
            try:
                conn, _ = self._server_.accept()
            except OSError:
                return
            n += 1
            self._conns_[n] = conn
            t = threading.Thread(target=self._serve, args=(n, conn),
                                 daemon=True)
            t.start()
            self._threads_.append(t)

    def _serve(self, cid, conn):
        while True:
            frame = recv_frame(conn)
            if frame is None:
                self._conns_.pop(cid, None)
                conn.close()
                return
            self.receive_data(cid, numpy.load(io.BytesIO(frame),
                                              allow_pickle=False))

    def receive_data(self, cid, data):
        self._queue_.put((cid, data))

    def reply(self, cid, result):
        conn = self._conns_.get(cid)
        if conn is None:
            return
        send_frame(conn, json.dumps(result, cls=NumpyJSONEncoder).encode())

    # --------------------------------------------------------------- unit
    def run(self):
        if self.cid is not None:
            fn = self.reply_fn or (lambda wf: wf.generate_data_for_master())
            self.reply(self.cid, fn(self.workflow))
        self.cid, self.output = self._queue_.get()

    def stop(self):
        self.receive_data(None, None)
        if self._server_ is not None:
            try:
                self._server_.close()
            except OSError:
                pass

    # ------------------------------------------------------ IDistributable
    def generate_data_for_master(self):
        return {"QueueLoaderEndpoints": dict(self.endpoints)}

    def generate_data_for_slave(self, slave=None):
        return None

    def apply_data_from_master(self, data):
        pass

    def apply_data_from_slave(self, data, slave=None):
        if data:
            key = getattr(slave, "id", slave)
            self.endpoints[key] = data.get("QueueLoaderEndpoints")

    def drop_slave(self, slave=None):
        self.endpoints.pop(getattr(slave, "id", slave), None)

    def __getstate__(self):
        st = super().__getstate__()
        st["reply_fn"] = None
        st["output"] = None
        st["cid"] = None
        return st


class QueueLoaderClient(object):
    """``QueueLoaderClient(loader.endpoints).request(array) -> reply``."""

    def __init__(self, endpoints):
        if "ipc" in endpoints:
            self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            self.sock.connect(endpoints["ipc"])
        else:
            host, port = endpoints["tcp"].rsplit(":", 1)
            self.sock = socket.create_connection((host, int(port)))

    def send(self, array):
        buf = io.BytesIO()
        numpy.save(buf, numpy.asarray(array), allow_pickle=False)
        send_frame(self.sock, buf.getvalue())

    def receive(self):
        frame = recv_frame(self.sock)
        return None if frame is None else json.loads(frame.decode())

    def request(self, array):
        self.send(array)
        return self.receive()

    def close(self):
        self.sock.close()
