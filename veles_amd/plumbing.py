"""Control-flow service units (reference: veles/plumbing.py:17-112)."""
from __future__ import annotations

from veles_amd.distributable import TriviallyDistributable
from veles_amd.units import TrivialUnit, Unit

__all__ = ["Repeater", "StartPoint", "EndPoint", "FireStarter",
           "UttermostPoint"]


class Repeater(TrivialUnit):
    """Closes a control-flow cycle; fires on any single notification."""

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "PLUMBING")
        kwargs["ignore_gate"] = True
        super().__init__(workflow, **kwargs)

    def link_from(self, *args):
        super().link_from(*args)
        if len(self.links_from) > 2:
            self.warning("Repeater has more than 2 incoming links: %s. Are "
                         "you sure?", [u.name for u in self.links_from])
        return self


class UttermostPoint(TrivialUnit):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)

    @property
    def name(self):
        wf = self.workflow
        base = self.__dict__.get("_name") or type(self).__name__
        if wf is not None:
            return "%s of %s" % (base, type(wf).__name__)
        return base

    @name.setter
    def name(self, value):
        self._name = value


class StartPoint(UttermostPoint):
    """Workflow execution starts here."""
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("name", "Start")
        super().__init__(workflow, **kwargs)


class _Deferred(object):
    """A scheduler entry that calls ``fn`` when its turn comes."""
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn

    def _check_gate_and_run(self, src):
        self.fn()


class EndPoint(UttermostPoint):
    """Ends the pipeline; notifies the workflow that it finished."""
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("name", "End")
        super().__init__(workflow, **kwargs)

    def run(self):
        from veles_amd.units import _Scheduler
        sched = _Scheduler.current()
        if sched is None:
            self.workflow.on_workflow_finished()
            return
        # let the units already notified in this wave (siblings of the end
        # point, e.g. plotters of the final epoch) run before finishing
        sched.pending.append((_Deferred(self.workflow.on_workflow_finished),
                              self))

    def generate_data_for_master(self):
        return True

    def apply_data_from_slave(self, data, slave):
        if not self.gate_block:
            self.workflow.on_workflow_finished()


class FireStarter(Unit, TriviallyDistributable):
    """Resets ``stopped`` of the associated units."""

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "SERVICE")
        super().__init__(workflow, **kwargs)
        self._units = set(kwargs.get("units", ()))

    @property
    def units(self):
        return self._units

    def initialize(self, **kwargs):
        pass

    def run(self):
        for unit in self._units:
            unit.stopped = False
