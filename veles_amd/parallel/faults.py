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

__all__ = ["FaultInjector", "Watchdog", "hook_decision"]


def hook_decision(workflow, after):
    """Call ``after()`` each time the workflow's decision unit has run (one
    run per minibatch).  The scheduler dispatches a unit through its
    ``do_run`` (units.py ``_check_gate_and_run``), and a direct ``run()``
    goes through the same bound method, so both instance entries are
    replaced by one wrapper.  Returns False when there is no decision."""
    dec = getattr(workflow, "decision", None)
    if dec is None:
        return False
    name = "do_run" if hasattr(dec, "do_run") else "run"
    orig = getattr(dec, name)

    def run_then():
        orig()
        after()
    dec.__dict__[name] = run_then
    if name == "do_run":
        dec.__dict__["run"] = run_then
    return True


class FaultInjector(object):
    EXIT_CODE = 75

    def __init__(self, workflow, probability, seed=None):
        self.workflow = workflow
        self.p = float(probability)
        self.rng = random.Random(seed if seed is not None else os.getpid())

    def install(self):
        inj = self

        def maybe_die():
            if inj.rng.random() < inj.p:
                print("[fault] injected death of rank %s" %
                      os.environ.get("RANK", "0"), file=sys.stderr,
                      flush=True)
                os._exit(FaultInjector.EXIT_CODE)
        hook_decision(self.workflow, maybe_die)
        return self


class Watchdog(object):
    """Exit a rank whose training step stops making progress.

    ``timeout``: the longest allowed gap between two kicks (decision runs,
    one per minibatch).  ``init_timeout`` (optional): the step limit is then
    ARMED by the first kick only - the first step (kernel loading, HIP-graph
    capture, the first collectives) may take up to ``init_timeout`` seconds
    from ``start``, and every later step ``timeout`` - so that a short
    per-step bound does not fire during initialisation (bench.py: 300 s to
    the first step, 60 s per step after it, both below the driver's 600 s
    limit on the whole command)."""

    def __init__(self, timeout, on_expire=None, init_timeout=None):
        self.timeout = float(timeout)
        self.init_timeout = None if init_timeout is None else \
            float(init_timeout)
        self.on_expire = on_expire or (lambda: os._exit(124))
        self._last = time.time()
        self._armed = init_timeout is None
        self.kicks = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True)

    def start(self):
        self._last = time.time()
        self._t.start()
        return self

    def kick(self):
        self._last = time.time()
        self.kicks += 1
        self._armed = True

    @property
    def armed(self):
        return self._armed

    def install(self, workflow):
        """Kick on every decision run (one per minibatch): a rank whose step
        stalls longer than ``timeout`` exits 124 so the launcher can respawn
        the group (the reference's per-slave job timeout, server.py:619-635,
        ``--job-timeout``)."""
        if not hook_decision(workflow, self.kick):
            return self
        return self.start()

    def stop(self):
        self._stop.set()

    def _limit(self):
        return self.timeout if self._armed else self.init_timeout

    def _loop(self):
        poll = min(1.0, self.timeout / 4, (self.init_timeout or 1.0) / 4)
        while not self._stop.wait(poll):
            limit = self._limit()
            if time.time() - self._last > limit:
                print("[watchdog] no progress for %.1f s (%s)" % (
                    limit, "per step" if self._armed else
                    "before the first step"), file=sys.stderr, flush=True)
                self.on_expire()
                return
