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
import contextlib
import os
import signal
import socket
import threading

from veles_amd.units import Unit
from veles_amd.utils.config import get, root

__all__ = ["Shell", "serve_console", "install_manhole"]


def serve_console(path, namespace):
    """Serve ONE Python console client on the UNIX socket ``path``."""
    try:
        os.remove(path)
    except OSError:
        pass
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(path)
    srv.listen(1)
    try:
        conn, _ = srv.accept()
        f = conn.makefile("rw")
        console = code.InteractiveConsole(namespace)
        console.write = lambda data: (f.write(data), f.flush())
        f.write(">>> ")
        f.flush()
        for line in f:
            # the client sees what the statement prints (stdout of the
            # process while it runs: this is a debugging console)
            with contextlib.redirect_stdout(f):
                more = console.push(line.rstrip("\n"))
            f.write("... " if more else ">>> ")
            f.flush()
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
    (``/tmp/veles_amd_manhole_<pid>.sock`` by default; ``nc -U`` it).
    Returns the socket path."""
    path = path or "/tmp/veles_amd_manhole_%d.sock" % os.getpid()

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
