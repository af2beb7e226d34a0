"""Interactive shell into a running workflow (reference
veles/interaction.py:49-95 IPython embed on a keypress, and the manhole
UNIX-socket REPL).

``Shell`` is a unit; when it runs and ``root.common.interactive`` is set, or
when the process receives SIGUSR2 (``install_signal``), it opens a Python
console (``code.interact``) with ``workflow`` / ``root`` / the unit in
scope.  With ``socket_path`` the console is served on a UNIX socket
instead (one client at a time), so a detached training run can be
inspected with ``nc -U``.
"""
from __future__ import annotations

import code
import os
import signal
import socket
import sys
import tempfile
import threading

from veles_amd.units import Unit
from veles_amd.utils.config import get, root

__all__ = ["Shell", "serve_console", "install_manhole"]


class _ThreadStdout(object):
    """sys.stdout proxy: writes from threads registered in ``sinks`` go to
    their sink (a console client), every other thread's to the original
    stream - so a console does not capture the training thread's output."""

    def __init__(self, orig):
        self.orig = orig
        self.sinks = {}

    def _target(self):
        return self.sinks.get(threading.get_ident(), self.orig)

    def write(self, data):
        return self._target().write(data)

    def flush(self):
        return self._target().flush()

    def __getattr__(self, name):
        return getattr(self.orig, name)


_stdout_lock = threading.Lock()


def _route_stdout(sink):
    with _stdout_lock:
        if not isinstance(sys.stdout, _ThreadStdout):
            sys.stdout = _ThreadStdout(sys.stdout)
        sys.stdout.sinks[threading.get_ident()] = sink


def _unroute_stdout():
    with _stdout_lock:
        if isinstance(sys.stdout, _ThreadStdout):
            sys.stdout.sinks.pop(threading.get_ident(), None)


def serve_console(path, namespace):
    """Serve ONE Python console client on the UNIX socket ``path``.  The
    socket is created owner-only (mode 0600) whatever the umask; ``path``
    must not exist yet (a path in a shared directory that someone else
    created is never removed or reused)."""
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    old = os.umask(0o177)
    try:
        srv.bind(path)
    finally:
        os.umask(old)
    os.chmod(path, 0o600)
    srv.listen(1)
    try:
        conn, _ = srv.accept()
        f = conn.makefile("rw")
        console = code.InteractiveConsole(namespace)
        console.write = lambda data: (f.write(data), f.flush())
        f.write(">>> ")
        f.flush()
        # what a statement prints goes to the client; other threads keep
        # the process's stdout
        _route_stdout(f)
        try:
            for line in f:
                more = console.push(line.rstrip("\n"))
                f.write("... " if more else ">>> ")
                f.flush()
        finally:
            _unroute_stdout()
        conn.close()
    finally:
        srv.close()
        try:
            os.remove(path)
        except OSError:
            pass


def install_manhole(workflow, path=None):
    """``--manhole`` (reference thread_pool.py:139-142): on SIGUSR2 the
    process starts serving a console into ``workflow`` on a UNIX socket
    (``manhole.sock`` in a fresh owner-only directory by default; ``nc -U``
    it).  Returns the socket path."""
    if path is None:
        path = os.path.join(tempfile.mkdtemp(prefix="veles_amd_manhole_"),
                            "manhole.sock")

    def handler(signum, frame):
        ns = {"workflow": workflow, "root": root,
              "units": {u.name: u for u in workflow}}
        threading.Thread(target=serve_console, args=(path, ns),
                         daemon=True, name="manhole").start()
    signal.signal(signal.SIGUSR2, handler)
    return path


class Shell(Unit):
    MAPPING = "shell"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self.socket_path = kwargs.get("socket_path")

    def init_unpickled(self):
        super().init_unpickled()
        self.requested_ = False

    def namespace(self):
        return {"workflow": self.workflow, "root": root, "shell": self,
                "units": {u.name: u for u in self.workflow}}

    def install_signal(self):
        def handler(signum, frame):
            self.requested_ = True
        signal.signal(signal.SIGUSR2, handler)

    def run(self):
        if not (self.requested_ or get(root.common.interactive, False)):
            return
        self.requested_ = False
        if self.socket_path:
            threading.Thread(target=self.serve_socket, daemon=True).start()
        else:
            code.interact(banner="veles_amd shell (Ctrl-D to resume)",
                          local=self.namespace())

    def serve_socket(self):
        serve_console(self.socket_path, self.namespace())
