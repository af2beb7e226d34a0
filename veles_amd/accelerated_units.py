"""Device-backed units.

Reference: veles/accelerated_units.py:128-866 (``AcceleratedUnit`` with
ocl_/cuda_/numpy_ method triples, run-time kernel source generation and a
binary cache; ``DeviceBenchmark``; ``AcceleratedWorkflow`` with a cached
``computing_power``).

Here a unit has ONE ``run()``: it calls ``veles_amd.ops`` on torch tensors,
which dispatch to the precompiled gfx950 kernels for HIP tensors and to the
float32 reference for CPU tensors.  ``--force-cpu Unit1,Unit2`` pins units to
the CPU device (the reference's ``--force-numpy``); ``--sync-run`` synchronises
after every run so unit timers measure device time.
"""
from __future__ import annotations

import time

from veles_amd.backends import CpuDevice, Device
from veles_amd.units import Unit
from veles_amd.utils.config import root, get
from veles_amd.workflow import Workflow

__all__ = ["AcceleratedUnit", "TrivialAcceleratedUnit", "DeviceBenchmark",
           "AcceleratedWorkflow"]

_CPU = None


def cpu_device():
    global _CPU
    if _CPU is None:
        _CPU = CpuDevice()
    return _CPU


class AcceleratedUnit(Unit):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.force_cpu = kwargs.get("force_cpu", False)

    def init_unpickled(self):
        super().init_unpickled()
        self.device_ = None

    @property
    def device(self):
        return self.device_

    @device.setter
    def device(self, value):
        self.device_ = value

    @property
    def is_gpu(self):
        return bool(self.device_ is not None and self.device_.is_gpu)

    @property
    def torch_device(self):
        import torch
        d = self.device_
        return d.torch_device if d is not None else torch.device("cpu")

    @property
    def compute_dtype(self):
        import torch
        d = self.device_
        return d.compute_dtype if d is not None else torch.float32

    def initialize(self, device=None, **kwargs):
        forced = get(root.common.engine.force_cpu, ()) or ()
        if isinstance(forced, str):
            forced = forced.split(",")
        if self.force_cpu or type(self).__name__ in forced or \
                self.name in forced:
            device = cpu_device()
        if device is None:
            device = cpu_device()
        self.device_ = device

    def do_run(self):
        super().do_run()
        if get(root.common.engine.sync_run, False) and self.is_gpu:
            self.device_.sync()

    def init_vectors(self, *arrays):
        for a in arrays:
            if a is not None and a.mem is not None:
                a.initialize(self.device_)

    def unmap_vectors(self, *arrays):
        for a in arrays:
            if a is not None:
                a.unmap()


class TrivialAcceleratedUnit(AcceleratedUnit):
    def run(self):
        pass


class DeviceBenchmark(AcceleratedUnit):
    """C = A*B square GEMM timing (reference accelerated_units.py:705-824);
    returns ``1000/dt`` ("computing power") or the mean seconds.

    ``dtype`` "float32" / "float64" times the exact-precision MFMA SGEMM /
    DGEMM at ``precision_level`` 0/1/2 - the reference's only published
    device numbers are SGEMM/DGEMM 3001^3 at these levels
    (devices/device_infos.json); default: the device compute
    dtype (bf16 MFMA GEMM on the MI355X)."""

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.size = int(kwargs.get("size", 1500))
        self.repeats = int(kwargs.get("repeats", 10))
        self.dry_run_first = kwargs.get("dry_run_first", True)
        self.return_time = kwargs.get("return_time", False)
        self.dtype = kwargs.get("dtype")
        self.precision_level = kwargs.get("precision_level")

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        import torch
        n = self.size
        g = torch.Generator().manual_seed(1)
        a = torch.rand(n, n, generator=g, dtype=torch.float64) - 0.5
        b = torch.rand(n, n, generator=g, dtype=torch.float64) - 0.5
        dt = getattr(torch, self.dtype) if self.dtype else self.compute_dtype
        self.a_ = a.to(self.torch_device, dt)
        self.b_ = b.to(self.torch_device, dt)
        self.c_ = torch.empty(n, n, dtype=dt, device=self.torch_device)

    def _gemm(self):
        from veles_amd import ops
        kw = {}
        if self.a_.dtype in (torch_f32(), torch_f64()):
            kw["precision_level"] = self.precision_level
        ops.gemm(self.a_, self.b_, out=self.c_, **kw)

    def run(self):
        if self.dry_run_first:
            self._gemm()
        if self.is_gpu:
            self.device_.sync()
        t0 = time.perf_counter()
        for _ in range(self.repeats):
            self._gemm()
        if self.is_gpu:
            self.device_.sync()
        dt = (time.perf_counter() - t0) / self.repeats
        self.seconds = dt
        self.gflops = 2.0 * self.size ** 3 / dt / 1e9
        return dt if self.return_time else 1000.0 / dt


def torch_f32():
    import torch
    return torch.float32


def torch_f64():
    import torch
    return torch.float64


class AcceleratedWorkflow(Workflow):
    """Workflow owning a device; ``computing_power`` is cached for 120 s."""

    hide_from_registry = True

    def init_unpickled(self):
        super().init_unpickled()
        self._power_ = None
        self._power_time_ = 0.0

    def initialize(self, **kwargs):
        dev = kwargs.get("device")
        if dev is None and self.device is None:
            kwargs["device"] = Device()
        return super().initialize(**kwargs)

    @property
    def computing_power(self):
        now = time.time()
        if self._power_ is None or now - self._power_time_ > 120:
            from veles_amd.dummy import DummyWorkflow
            bench = DeviceBenchmark(DummyWorkflow(), size=1024, repeats=3)
            bench.initialize(device=self.device)
            self._power_ = bench.run()
            self._power_time_ = now
        return self._power_
