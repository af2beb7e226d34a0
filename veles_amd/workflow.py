"""Workflow: a container unit owning a graph of units.

Reference: veles/workflow.py:86-1051.  Behaviour kept: units keyed by name
(a multimap), dependency-ordered ``initialize`` with retry, ``run`` from
``start_point`` to ``EndPoint``, aggregated distributed hooks, Graphviz DOT
graph, per-unit timing statistics, ``--result-file`` JSON from
``IResultProvider`` units, the source-file checksum and ``package_export``
(zip / tgz with ``contents.json`` + ``NNNN_AxB.npy``) consumed by the native
runtime (csrc/runtime).

MI355X specifics: ``run()`` enqueues every unit's kernels on the device's
compute HIP stream (``device.stream()``), so the whole step is stream-ordered
and may be captured into a HIP graph (``veles_amd.parallel.graphs``).
"""
from __future__ import annotations

import hashlib
import inspect
import io
import json
import os
import sys
import tarfile
import time
import zipfile
from collections import OrderedDict

import numpy

from veles_amd.error import VelesException
from veles_amd.plumbing import EndPoint, Repeater, StartPoint
from veles_amd.thread_pool import ThreadPool
from veles_amd.units import Container, Unit, _Scheduler
from veles_amd.utils.config import root, get
from veles_amd.utils.logger import events

__all__ = ["Workflow", "NoMoreJobs", "IResultProvider"]


class NoMoreJobs(Exception):
    pass


class IResultProvider(object):
    """Units that contribute metrics to the results file
    (reference veles/result_provider.py:41-58)."""

    def get_metric_names(self):
        raise NotImplementedError

    def get_metric_values(self):
        raise NotImplementedError


class Workflow(Container):
    hide_from_registry = True

    VIEW_GROUP_COLORS = {"PLOTTER": "gold", "WORKER": "greenyellow",
                         "LOADER": "cyan", "TRAINER": "coral",
                         "EVALUATOR": "plum", "SERVICE": "lightgrey",
                         "PLUMBING": "white"}

    def __init__(self, workflow, **kwargs):
        self._units = []
        self._checksum = None
        self._restored_from_snapshot = False
        self._result_file = kwargs.get("result_file")
        super().__init__(workflow, **kwargs)
        self.start_point = StartPoint(self)
        self.end_point = EndPoint(self)

    def init_unpickled(self):
        super().init_unpickled()
        self._thread_pool_ = None
        self._finished_ = False
        self._run_time_started_ = None
        self._run_time_ = 0.0
        self.device_ = None

    def __setstate__(self, state):
        super().__setstate__(state)
        self._restored_from_snapshot = True

    @property
    def device(self):
        dev = self.__dict__.get("device_")
        if dev is None:
            parent = self.__dict__.get("_workflow")
            if parent is not None and parent is not self:
                dev = getattr(parent, "device", None)
        return dev

    @device.setter
    def device(self, value):
        self.device_ = value

    # -- container protocol ---------------------------------------------
    def add_ref(self, unit):
        if unit is self:
            raise ValueError("Attempted to add self to self")
        if unit not in self._units:
            self._units.append(unit)
        self._checksum = None

    def del_ref(self, unit):
        if unit in self._units:
            self._units.remove(unit)
        self._checksum = None

    def __iter__(self):
        return iter(list(self._units))

    def __len__(self):
        return len(self._units)

    def __contains__(self, unit):
        return unit in self._units

    def index_of(self, unit):
        return self._units.index(unit)

    def __getitem__(self, key):
        if isinstance(key, int):
            return self._units[key]
        if isinstance(key, str):
            found = [u for u in self._units if u.name == key]
            if not found:
                raise KeyError(key)
            return found[0] if len(found) == 1 else found
        raise TypeError(key)

    @property
    def units(self):
        return list(self._units)

    @property
    def units_in_dependency_order(self):
        order = list(self.start_point.dependent_units())
        seen = set(order)
        for u in self._units:
            if u not in seen:
                order.append(u)
        return order

    @property
    def restored_from_snapshot(self):
        return self._restored_from_snapshot

    @property
    def is_master(self):
        return bool(getattr(self.workflow, "is_master", False))

    @property
    def is_slave(self):
        return bool(getattr(self.workflow, "is_slave", False))

    @property
    def is_standalone(self):
        return bool(getattr(self.workflow, "is_standalone", True))

    @property
    def interactive(self):
        return bool(getattr(self.workflow, "interactive", False))

    @property
    def thread_pool(self):
        if self._thread_pool_ is None:
            parent = self.workflow
            pool = getattr(parent, "thread_pool", None) if not isinstance(
                parent, Workflow) or parent is not self else None
            if not isinstance(pool, ThreadPool):
                pool = ThreadPool(
                    get(root.common.engine.thread_pool.minthreads, 2),
                    get(root.common.engine.thread_pool.maxthreads, 2),
                    name=self.name)
            self._thread_pool_ = pool
        return self._thread_pool_

    # -- lifecycle ----------------------------------------------------------
    def initialize(self, **kwargs):
        """Initialize units in dependency (BFS) order; units returning True
        are retried after the others (reference workflow.py:303-349)."""
        device = kwargs.get("device")
        if device is not None:
            self.device = device
        elif self.device is None:
            self.device = getattr(self.workflow, "device", None)
        kwargs["device"] = self.device
        pending = list(self.units_in_dependency_order)
        # a re-initialized workflow runs again (FireStarter semantics)
        self._finished_ = False
        for u in pending:
            if u is not self:
                u.stopped = False
        if self._restored_from_snapshot:
            for u in pending:
                if not getattr(u, "_remembers_gates", True):
                    u.gate_block <<= False
                    u.gate_skip <<= False
        retries = 0
        while pending:
            unit = pending.pop(0)
            if unit is self:
                continue
            retry = unit.initialize(**kwargs)
            if retry:
                pending.append(unit)
                retries += 1
                if retries > 10 * (len(self._units) + 1):
                    raise VelesException(
                        "Unit %s keeps requesting initialize() retries" %
                        unit)
        return None

    def run(self):
        """Run the graph from start_point until it drains."""
        if self.is_master:
            # rank 0 of a job-farm does not compute; see parallel.jobfarm
            return
        self._finished_ = False
        self._run_time_started_ = time.perf_counter()
        self.event("run", "begin")
        ctx = None
        dev = self.device
        if dev is not None and getattr(dev, "is_gpu", False):
            import torch
            ctx = torch.cuda.stream(dev.stream())
            ctx.__enter__()
        try:
            with _Scheduler() as sched:
                self.start_point.run_dependent()
                sched.drain()
        finally:
            if ctx is not None:
                ctx.__exit__(None, None, None)
            self._run_time_ += time.perf_counter() - self._run_time_started_
            self.event("run", "end")

    def stop(self):
        for unit in self._units:
            if unit is not self:
                try:
                    unit.stop()
                except Exception:
                    self.exception("Failed to stop %s", unit)

    def on_workflow_finished(self):
        self._finished_ = True
        for unit in self._units:
            if unit is not self:
                unit.stopped = True
        if self._result_file:
            self.write_results(self._result_file)
        parent = self.workflow
        cb = getattr(parent, "on_workflow_finished", None)
        if cb is not None and parent is not self:
            cb()

    @property
    def finished(self):
        return self._finished_

    def del_units(self):
        for u in list(self._units):
            u.unlink_all()
        self._units = []

    def change_unit(self, name, new_unit):
        """Replace the unit called ``name`` keeping its control links
        (reference workflow.py:977-1051)."""
        old = self[name]
        if isinstance(old, list):
            raise ValueError("Ambiguous unit name %s" % name)
        froms = list(old.links_from)
        tos = list(old.links_to)
        old.unlink_all()
        for s in froms:
            new_unit.link_from(s)
        for d in tos:
            d.link_from(new_unit)
        self.del_ref(old)
        if new_unit.workflow is not self:
            new_unit.workflow = self
        return new_unit

    # -- distributed hooks (aggregate over units in dependency order) ------
    def generate_initial_data_for_slave(self, slave=None):
        return [getattr(u, "generate_initial_data_for_slave",
                        lambda s: None)(slave)
                for u in self.units_in_dependency_order if u is not self]

    def apply_initial_data_from_master(self, data):
        units = [u for u in self.units_in_dependency_order if u is not self]
        for u, d in zip(units, data):
            fn = getattr(u, "apply_initial_data_from_master", None)
            if fn is not None and d is not None:
                fn(d)

    def generate_data_for_slave(self, slave=None):
        self.event("generate_data", "begin")
        out = []
        for u in self.units_in_dependency_order:
            if u is self:
                continue
            try:
                out.append(u.generate_data_for_slave(slave))
            except NoMoreJobs:
                self.event("generate_data", "end")
                return None
        self.event("generate_data", "end")
        return out

    def generate_data_for_master(self):
        return [u.generate_data_for_master()
                for u in self.units_in_dependency_order if u is not self]

    def apply_data_from_master(self, data):
        units = [u for u in self.units_in_dependency_order if u is not self]
        for u, d in zip(units, data):
            u.apply_data_from_master(d)

    def apply_data_from_slave(self, data, slave=None):
        units = [u for u in self.units_in_dependency_order if u is not self]
        for u, d in zip(units, data):
            u.apply_data_from_slave(d, slave)

    def drop_slave(self, slave=None):
        for u in self._units:
            if u is not self:
                u.drop_slave(slave)

    def do_job(self, data, update=None, callback=None):
        """Execute one job received from rank 0 (reference workflow.py:558)."""
        self.apply_data_from_master(data)
        self.run()
        result = self.generate_data_for_master()
        if callback is not None:
            callback(result)
        return result

    # -- introspection ------------------------------------------------------
    def generate_graph(self, filename=None, write_on_disk=True,
                       with_data_links=False, quiet=True):
        """Graphviz DOT of the control flow (and optional data links)."""
        lines = ["digraph Workflow {",
                 '  bgcolor="transparent"; mindist=0.5; overlap="false";']
        ids = {}
        order = self.units_in_dependency_order
        for i, u in enumerate(order):
            if u is self:
                continue
            ids[u] = "u%d" % i
            try:
                fname = os.path.relpath(inspect.getfile(type(u)),
                                        root.common.dirs.veles)
            except Exception:
                fname = "?"
            color = self.VIEW_GROUP_COLORS.get(u.view_group, "white")
            lines.append(
                '  %s [label=<<b>%s</b><br/><font point-size="10">%s</font>>'
                ', shape=rect, style="rounded,filled", fillcolor="%s"];' %
                (ids[u], _html(u.name), _html(fname), color))
        for u in order:
            if u not in ids:
                continue
            for d in u.links_to_sorted:
                if d in ids:
                    lines.append("  %s -> %s [penwidth=3];" % (ids[u], ids[d]))
        if with_data_links:
            for u in order:
                if u not in ids:
                    continue
                for k, v in u.__dict__.items():
                    if k.startswith("_lnk_") and v[0] in ids:
                        lines.append(
                            '  %s -> %s [style=dashed, color=gray, '
                            'label="%s", constraint=false];' %
                            (ids[u], ids[v[0]], k[5:] if k[5:] == v[1]
                             else "%s <- %s" % (k[5:], v[1])))
        lines.append("}")
        desc = "\n".join(lines)
        if write_on_disk and filename:
            with open(filename, "w") as f:
                f.write(desc)
        return desc, filename

    def get_unit_run_time_stats(self, by_name=False):
        stats = []
        for u in self._units:
            if u is self:
                continue
            stats.append((u.name if by_name else u, u.total_run_time,
                          u._run_calls))
        stats.sort(key=lambda x: -x[1])
        return stats

    def print_stats(self, by_name=False, top_number=5, file=None):
        file = file or sys.stdout
        stats = self.get_unit_run_time_stats()
        total = sum(s[1] for s in stats) or 1e-12
        print("Unit run time statistics top %d:" % top_number, file=file)
        print("%-36s %10s %8s %7s" % ("unit", "time s", "calls", "%"),
              file=file)
        for u, t, n in stats[:top_number]:
            print("%-36s %10.4f %8d %6.1f%%" % (u.name[:36], t, n,
                                                100.0 * t / total), file=file)
        wall = self._run_time_
        if wall > 0:
            print("Workflow wall time %.4f s, unit time %.4f s (%.1f%% "
                  "efficiency)" % (wall, total, 100.0 * total / wall),
                  file=file)

    def gather_results(self):
        results = {"id": getattr(self.workflow, "id", None),
                   "log_id": getattr(self.workflow, "log_id", None)}
        for u in self._units:
            if hasattr(u, "get_metric_values") and u is not self:
                try:
                    results.update(u.get_metric_values())
                except NotImplementedError:
                    pass
        return results

    def write_results(self, file=None):
        file = file or self._result_file
        results = self.gather_results()
        from veles_amd.utils.json_encoders import NumpyJSONEncoder
        if hasattr(file, "write"):
            json.dump(results, file, cls=NumpyJSONEncoder, indent=2,
                      sort_keys=True)
        else:
            with open(file, "w") as f:
                json.dump(results, f, cls=NumpyJSONEncoder, indent=2,
                          sort_keys=True)
        return results

    @property
    def checksum(self):
        """sha1(source of the workflow's module) + "_" + len(units)
        (reference workflow.py:851-866)."""
        if self._checksum is None:
            sha1 = hashlib.sha1()
            mod = sys.modules.get(type(self).__module__)
            path = getattr(mod, "__file__", None)
            if path and os.path.exists(path):
                with open(path, "rb") as f:
                    sha1.update(f.read())
            else:
                sha1.update(type(self).__qualname__.encode())
            self._checksum = sha1.hexdigest() + "_%d" % len(self)
        return self._checksum

    # -- export for the native runtime ------------------------------------
    def package_export(self, file_name, archive_format="zip", precision=32):
        if archive_format not in ("zip", "tgz"):
            raise ValueError("Only \"zip\" and \"tgz\" formats are supported "
                             "(got %s)" % archive_format)
        if precision not in (16, 32):
            raise ValueError("Only 16-bit and 32-bit floats are supported "
                             "(got %s)" % precision)
        exported = [u for u in self.units_in_dependency_order
                    if u is not self and hasattr(u, "package_export")]
        if not exported:
            raise ValueError("No units support export")
        arrays = []

        def fname(arr, idx, json_mode):
            name = "%04d_%s" % (idx, "x".join(map(str, arr.shape)))
            return "@" + name if json_mode else name + ".npy"

        def default(obj):
            if isinstance(obj, numpy.ndarray):
                arrays.append(obj)
                return fname(obj, len(arrays) - 1, True)
            if isinstance(obj, (numpy.integer,)):
                return int(obj)
            if isinstance(obj, (numpy.floating,)):
                return float(obj)
            raise TypeError("Cannot export %r" % type(obj))

        obj = {"workflow": type(self).__name__, "checksum": self.checksum,
               "units": []}
        for u in exported:
            obj["units"].append({
                "class": {"name": type(u).__name__,
                          "uuid": getattr(type(u), "__id__", "")},
                "data": u.package_export(),
                "links": [exported.index(d) for d in u.derefed_links_to()
                          if d in exported]})
        # connectivity / acyclicity check (reference workflow.py:895-910)
        fifo, seen = [0], set()
        while fifo:
            i = fifo.pop(0)
            seen.add(i)
            links = obj["units"][i]["links"]
            if not links and i < len(exported) - 1:
                raise VelesException("Unit %s is not connected to any other "
                                     "unit" % exported[i])
            for c in links:
                if c in seen:
                    raise VelesException("Cycles are not allowed (%s -> %s)" %
                                         (exported[i], exported[c]))
            fifo.extend(links)
        text = json.dumps(obj, indent=4, sort_keys=True, default=default)

        def npy_bytes(arr):
            bio = io.BytesIO()
            numpy.save(bio, arr.astype("float%d" % precision))
            return bio.getvalue()

        if archive_format == "zip":
            with zipfile.ZipFile(file_name, "w", zipfile.ZIP_DEFLATED) as z:
                z.writestr("contents.json", text)
                for i, arr in enumerate(arrays):
                    z.writestr(fname(arr, i, False), npy_bytes(arr))
        else:
            with tarfile.open(file_name, "w:gz") as tar:
                def add(name, data):
                    ti = tarfile.TarInfo(name)
                    ti.size = len(data)
                    ti.mode = 0o666
                    tar.addfile(ti, io.BytesIO(data))
                add("contents.json", text.encode())
                for i, arr in enumerate(arrays):
                    add(fname(arr, i, False), npy_bytes(arr))
        self.info("Exported package to %s", file_name)
        return file_name


def _html(s):
    return (str(s).replace("&", "&amp;").replace("<", "&lt;")
            .replace(">", "&gt;"))
