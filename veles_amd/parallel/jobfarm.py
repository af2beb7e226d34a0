"""Job farm: run independent workflow evaluations as child processes, one
per device, in parallel (the task-parallel modes: genetic hyper-parameter
search and ensembles).

Reference: the master hands chromosome / model indices to slaves as jobs
(veles/genetics/optimization_workflow.py:181-286,
veles/ensemble/base_workflow.py:101-127) over the ZeroMQ job protocol, and
each evaluation is a ``python -m veles ... --result-file`` subprocess.
MI355X-first: no master/slave network layer — one node, a worker thread per
GPU, each child pinned to its GPU with ``HIP_VISIBLE_DEVICES`` (288 GB per
GPU fits a whole model per worker), results read back from the
``--result-file`` JSON.  Without GPUs the workers are CPU processes.
"""
from __future__ import annotations

import json
import os
import queue
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

from veles_amd.utils.logger import Logger

__all__ = ["JobFarm", "Job", "veles_argv"]


def veles_argv(*args):
    """argv of a child ``python -m veles_amd`` run."""
    return [sys.executable, "-m", "veles_amd"] + [str(a) for a in args]


class Job(object):
    __slots__ = ("argv", "env", "tag", "result", "returncode", "log")

    def __init__(self, argv, env=None, tag=None):
        self.argv = list(argv)
        self.env = dict(env or {})
        self.tag = tag
        self.result = None
        self.returncode = None
        self.log = ""


class JobFarm(Logger):
    def __init__(self, devices=None, workers=None, timeout=None,
                 keep_logs=False):
        super().__init__()
        if devices is None:
            devices = self.detect_devices()
        self.devices = list(devices)
        # GPUs: one child per device; CPU: a few children, few threads each
        self.workers = workers or (len(self.devices) if self.devices else
                                   max(1, min(4, (os.cpu_count() or 2) // 2)))
        self.timeout = timeout
        self.keep_logs = keep_logs

    @staticmethod
    def detect_devices():
        vis = os.environ.get("HIP_VISIBLE_DEVICES") or \
            os.environ.get("CUDA_VISIBLE_DEVICES")
        if vis:
            return [d for d in vis.split(",") if d != ""]
        try:
            import torch
            n = torch.cuda.device_count()
        except Exception:
            n = 0
        return [str(i) for i in range(n)]

    def _run_one(self, job, slots):
        dev = slots.get()
        fd, res = tempfile.mkstemp(prefix="veles-job-", suffix=".json")
        os.close(fd)
        try:
            env = dict(os.environ)
            env.update(job.env)
            env.setdefault("PYTHONPATH", os.getcwd())
            if dev is not None:
                env["HIP_VISIBLE_DEVICES"] = dev
            else:
                env.setdefault("OMP_NUM_THREADS", "2")
            argv = list(job.argv)
            if "--result-file" not in argv:
                # the result file goes before the positional arguments
                argv[3:3] = ["--result-file", res]
            else:
                res = argv[argv.index("--result-file") + 1]
            self.debug("job %s on %s: %s", job.tag, dev, " ".join(argv))
            p = subprocess.run(argv, env=env, capture_output=True, text=True,
                               timeout=self.timeout)
            job.returncode = p.returncode
            job.log = (p.stdout + p.stderr)[-20000:] if self.keep_logs or \
                p.returncode else ""
            if p.returncode == 0:
                try:
                    with open(res) as f:
                        job.result = json.load(f)
                except (OSError, ValueError) as e:
                    self.error("job %s wrote no valid result: %s", job.tag, e)
            else:
                self.error("job %s failed (rc %d):\n%s", job.tag,
                           p.returncode, job.log[-3000:])
        except subprocess.TimeoutExpired:
            job.returncode = -1
            self.error("job %s timed out", job.tag)
        finally:
            slots.put(dev)
            try:
                os.remove(res)
            except OSError:
                pass
        return job

    def map(self, jobs):
        """Run every job; returns them (``result`` = parsed JSON or None)."""
        jobs = list(jobs)
        slots = queue.Queue()
        devs = self.devices or [None]
        for i in range(self.workers):
            slots.put(devs[i % len(devs)])
        with ThreadPoolExecutor(self.workers) as ex:
            return list(ex.map(lambda j: self._run_one(j, slots), jobs))
