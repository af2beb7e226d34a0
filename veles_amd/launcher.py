"""Launcher: process role, device and data-parallel group, run orchestration.

Reference: veles/launcher.py:99-906 (role detection standalone / master /
slave, Twisted reactor, device creation, remote node spawning, status,
stats at shutdown, ``--result-file``).  Roles become ranks of a
``torch.distributed`` group: ``WORLD_SIZE > 1`` in the environment (set by
``veles_amd.parallel.launch`` or ``torch.distributed.run``) makes this a
data-parallel rank; rank 0 is the "master" for snapshots / results.  There
is no reactor: the calling thread runs the workflow.
"""
from __future__ import annotations

import os
import time
import uuid

from veles_amd.backends import Device
from veles_amd.utils.config import root
from veles_amd.utils.logger import Logger, events

__all__ = ["Launcher"]


class Launcher(Logger):
    is_launcher = True

    def __init__(self, backend="auto", device_id=None, result_file=None,
                 testing=False, trace_events=None, **kwargs):
        super().__init__()
        self.id = str(uuid.uuid4())
        self.log_id = kwargs.get("log_id") or self.id
        self.backend = backend
        self.device_id = device_id
        self.result_file = result_file
        self.testing = testing
        self.trace_events = trace_events
        self.workflow = None
        self.device = None
        self.dp_ = None
        self.snapshot_file = kwargs.get("snapshot_file")
        self.stopped = False
        self.start_time = time.time()
        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))

    def __getstate__(self):
        return {"id": self.id, "log_id": self.log_id, "testing": self.testing}

    def __setstate__(self, st):
        self.__dict__.update(st)
        self.dp_ = None
        self.device = None
        self.workflow = None

    # role properties used by units
    @property
    def is_master(self):
        return False  # sync DP: every rank computes

    @property
    def is_slave(self):
        return False

    @property
    def is_standalone(self):
        return True

    @property
    def is_rank0(self):
        return self.rank == 0

    @property
    def interactive(self):
        return False

    def add_ref(self, workflow):
        self.workflow = workflow

    def del_ref(self, unit):
        pass

    def initialize(self):
        if self.trace_events:
            events.enabled = True
        if self.world_size > 1 and self.dp_ is None:
            from veles_amd.parallel.dp import DataParallel
            be = "gloo" if self.backend in ("cpu", "numpy") else None
            from veles_amd.utils.config import root, get
            self.dp_ = DataParallel(backend=be, timeout_s=int(get(
                root.common.engine.dp.timeout_s, 600)))
        if self.device is None:
            kw = {}
            if self.device_id not in (None, ""):
                from veles_amd.backends import parse_device_spec
                ids = parse_device_spec(self.device_id)
                kw["device_id"] = ids[self.rank % len(ids)]
            self.device = Device(backend=self.backend, **kw)
        if self.dp_ is not None and self.snapshot_file:
            self._check_same_snapshot()
        self.info("rank %d/%d on %s", self.rank, self.world_size, self.device)
        return self.device

    def _check_same_snapshot(self):
        """Every rank of a resumed data-parallel job must have restored the
        same snapshot bytes: replicas that resume different epochs / loader
        positions / momenta diverge and deadlock at the next epoch end."""
        import os
        from veles_amd.parallel.launch import snapshot_digest
        from veles_amd.snapshotter import loaded_digest
        # the bytes this rank restored (import_snapshot records the row /
        # download it loaded: a sqlite:// spec without a row id names the
        # NEWEST row, which differs between ranks while a snapshotter
        # writes or across nodes)
        got = loaded_digest(self.snapshot_file)
        if got is not None:
            mine = tuple(got[:2])
        elif os.path.isfile(self.snapshot_file):
            mine = snapshot_digest(self.snapshot_file)
        else:
            raise RuntimeError(
                "cannot tell which snapshot bytes %r restored on rank %d" %
                (self.snapshot_file, self.rank))
        allv = self.dp_.all_gather_object(mine)
        if any(v != allv[0] for v in allv):
            raise RuntimeError(
                "ranks resumed from different snapshots %s (this rank: %s); "
                "a multi-node job needs a shared snapshot directory" %
                (allv, self.snapshot_file))

    def run(self):
        wf = self.workflow
        t0 = time.time()
        wf.run()
        self.info("Workflow finished in %.2f s", time.time() - t0)

    def on_workflow_finished(self):
        self.stopped = True

    def finish(self):
        wf = self.workflow
        if wf is not None and self.rank == 0:
            try:
                wf.print_stats()
            except Exception:
                pass
            if self.result_file:
                wf.write_results(self.result_file)
        if self.trace_events:
            path = self.trace_events
            if self.world_size > 1:
                base, ext = os.path.splitext(path)
                path = "%s.rank%d%s" % (base, self.rank, ext or ".json")
            events.dump(path)
        if self.dp_ is not None:
            self.dp_.barrier()

    def stop(self):
        if self.workflow is not None:
            self.workflow.stop()
        self.stopped = True
