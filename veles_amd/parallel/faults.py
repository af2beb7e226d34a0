"""Fault injection and failure detection for data-parallel runs.

Reference: ``--slave-death-probability`` (veles/client.py:303-307, 438-442)
and the master's job-timeout / hang detection (server.py:385-394, 619-635).
``FaultInjector`` kills this rank with probability p after each training
step (``os._exit``, as an abrupt process death would); ``Watchdog`` aborts a
rank whose step did not finish within ``timeout`` seconds so the launcher
can restart the group (collectives otherwise wait for their own timeout).
"""
from __future__ import annotations

import os
import random
import sys
import threading
import time

__all__ = ["FaultInjector", "Watchdog"]


class FaultInjector(object):
    EXIT_CODE = 75

    def __init__(self, workflow, probability, seed=None):
        self.workflow = workflow
        self.p = float(probability)
        self.rng = random.Random(seed if seed is not None else os.getpid())

    def install(self):
        dec = getattr(self.workflow, "decision", None)
        if dec is None:
            return self
        orig = dec.run
        inj = self

        def run_and_maybe_die():
            orig()
            if inj.rng.random() < inj.p:
                print("[fault] injected death of rank %s" %
                      os.environ.get("RANK", "0"), file=sys.stderr,
                      flush=True)
                os._exit(FaultInjector.EXIT_CODE)
        dec.__dict__["run"] = run_and_maybe_die
        return self


class Watchdog(object):
    def __init__(self, timeout, on_expire=None):
        self.timeout = timeout
        self.on_expire = on_expire or (lambda: os._exit(124))
        self._last = time.time()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True)

    def start(self):
        self._t.start()
        return self

    def kick(self):
        self._last = time.time()

    def install(self, workflow):
        """Kick on every decision run (one per minibatch): a rank whose step
        stalls longer than ``timeout`` exits 124 so the launcher can respawn
        the group (the reference's per-slave job timeout, server.py:619-635,
        ``--job-timeout``)."""
        dec = getattr(workflow, "decision", None)
        if dec is None:
            return self
        orig = dec.run
        wd = self

        def run_and_kick():
            orig()
            wd.kick()
        dec.__dict__["run"] = run_and_kick
        return self.start()

    def stop(self):
        self._stop.set()

    def _loop(self):
        while not self._stop.wait(min(1.0, self.timeout / 4)):
            if time.time() - self._last > self.timeout:
                print("[watchdog] no progress for %.1f s" % self.timeout,
                      file=sys.stderr, flush=True)
                self.on_expire()
                return
