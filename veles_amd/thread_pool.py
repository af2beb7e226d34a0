"""Worker thread pool for fan-out unit execution.

Reference: veles/thread_pool.py:70-608 (Twisted-based pool with pause/resume,
thread enter/exit hooks, shutdown hooks, SIGINT-safe shutdown, SIGUSR1 stack
dumps, failure capture).  Rebuilt on the stdlib; no reactor.  GPU work is
stream-ordered, so the pool only carries the *host* side of independent
branches (the HIP stream of the calling unit is captured per task).
"""
from __future__ import annotations

import logging
import queue
import signal
import sys
import threading
import traceback

__all__ = ["ThreadPool"]

_log = logging.getLogger("ThreadPool")


class ThreadPool(object):
    interrupted = False
    pools = []
    _sigusr1_installed = False

    def __init__(self, minthreads=2, maxthreads=2, name="pool"):
        self.min = max(0, int(minthreads))
        self.max = max(self.min, int(maxthreads), 1)
        self.name = name
        self._q = queue.Queue()
        self._threads = []
        self._lock = threading.Lock()
        self._paused = threading.Event()
        self._paused.set()
        self._idle = 0
        self.started = False
        self.joined = False
        self.failure = None
        self.on_thread_enter = []
        self.on_thread_exit = []
        self._shutdown_callbacks = []
        self._outstanding = 0
        self._done = threading.Condition(self._lock)
        ThreadPool.pools.append(self)
        ThreadPool._install_sigusr1()

    # -- lifecycle ----------------------------------------------------------
    def start(self):
        with self._lock:
            if self.started:
                return
            self.started = True
            self.joined = False
            for _ in range(self.min or 1):
                self._spawn()

    def _spawn(self):
        t = threading.Thread(target=self._worker,
                             name="%s-%d" % (self.name, len(self._threads)),
                             daemon=True)
        self._threads.append(t)
        t.start()

    def _worker(self):
        for cb in self.on_thread_enter:
            cb()
        try:
            while True:
                item = self._q.get()
                if item is None:
                    break
                self._paused.wait()
                fn, args, kwargs, callback = item
                try:
                    res = fn(*args, **kwargs)
                    ok = True
                except BaseException as e:  # noqa
                    res = e
                    ok = False
                    self.failure = (e, traceback.format_exc())
                    _log.error("Task %s failed:\n%s", fn, self.failure[1])
                if callback is not None:
                    try:
                        callback(ok, res)
                    except Exception:
                        _log.exception("callback failed")
                with self._lock:
                    self._outstanding -= 1
                    if self._outstanding == 0:
                        self._done.notify_all()
        finally:
            for cb in self.on_thread_exit:
                cb()

    def callInThread(self, fn, *args, **kwargs):
        self.callInThreadWithCallback(None, fn, *args, **kwargs)

    def callInThreadWithCallback(self, callback, fn, *args, **kwargs):
        if self.joined:
            raise RuntimeError("ThreadPool %s is shut down" % self.name)
        if not self.started:
            self.start()
        with self._lock:
            self._outstanding += 1
            busy = self._outstanding
            if busy > len(self._threads) and len(self._threads) < self.max:
                self._spawn()
        self._q.put((fn, args, kwargs, callback))

    def wait_idle(self, timeout=None):
        with self._lock:
            if self._outstanding == 0:
                return True
            return self._done.wait_for(lambda: self._outstanding == 0,
                                       timeout)

    def pause(self):
        self._paused.clear()

    def resume(self):
        self._paused.set()

    def register_on_shutdown(self, fn):
        self._shutdown_callbacks.append(fn)

    def shutdown(self, timeout=10.0):
        if self.joined:
            return
        for cb in list(self._shutdown_callbacks):
            try:
                cb()
            except Exception:
                _log.exception("shutdown callback failed")
        self._paused.set()
        with self._lock:
            threads = list(self._threads)
            self.joined = True
        for _ in threads:
            self._q.put(None)
        for t in threads:
            if t is not threading.current_thread():
                t.join(timeout)
        self._threads = []
        self.started = False
        if self in ThreadPool.pools:
            ThreadPool.pools.remove(self)

    @staticmethod
    def shutdown_pools():
        for p in list(ThreadPool.pools):
            p.shutdown()

    # -- debugging ----------------------------------------------------------
    @staticmethod
    def _install_sigusr1():
        if ThreadPool._sigusr1_installed:
            return
        if threading.current_thread() is not threading.main_thread():
            return
        try:
            signal.signal(signal.SIGUSR1, ThreadPool.sigusr1_handler)
            ThreadPool._sigusr1_installed = True
        except (ValueError, OSError, AttributeError):
            pass

    @staticmethod
    def sigusr1_handler(signum=None, frame=None):
        """Dump every thread's stack (reference thread_pool.py:520-525)."""
        print(ThreadPool.format_stacks(), file=sys.stderr)

    @staticmethod
    def format_stacks():
        out = []
        names = {t.ident: t.name for t in threading.enumerate()}
        for tid, frame in sys._current_frames().items():
            out.append("--- thread %s (%s) ---" % (names.get(tid, "?"), tid))
            out.extend(traceback.format_stack(frame))
        return "\n".join(out)
