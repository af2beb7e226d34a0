"""Test / benchmark harness (reference veles/dummy.py:46-131)."""
from __future__ import annotations

import time
import uuid

from veles_amd.units import TrivialUnit
from veles_amd.workflow import Workflow

__all__ = ["DummyLauncher", "DummyWorkflow", "DummyUnit"]


class DummyLauncher(object):
    is_launcher = True

    def __init__(self, device=None):
        self.stopped = False
        self.testing = False
        self.id = str(uuid.uuid4())
        self.device = device
        self.workflow = None

    interactive = False
    is_slave = False
    is_master = False
    is_standalone = True
    log_id = "DUMMY"
    workflow_file = "/path/to/workflow"
    config_file = "/path/to/config"
    seeds = []

    @property
    def start_time(self):
        return time.time() - 1000

    def add_ref(self, workflow):
        self.workflow = workflow

    def __getstate__(self):
        # process-local handles (the data-parallel group ``dp_``, streams)
        # never enter a snapshot, as in Launcher.__getstate__
        return {k: v for k, v in self.__dict__.items()
                if not k.endswith("_")}

    def del_ref(self, unit):
        pass

    def on_workflow_finished(self):
        pass

    def stop(self):
        pass


class DummyWorkflow(Workflow):
    """Standalone workflow whose start point is pre-linked to its end."""

    def __init__(self, device=None):
        self._launcher = DummyLauncher(device)
        super().__init__(self._launcher)
        self.end_point.link_from(self.start_point)
        if device is not None:
            self.device = device

    @property
    def launcher(self):
        return self._launcher


class DummyUnit(TrivialUnit):
    disable_misprint_check = True

    def __init__(self, **kwargs):
        super().__init__(DummyWorkflow())
        self.__dict__.update(kwargs)
