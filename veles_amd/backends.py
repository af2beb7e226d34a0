"""Device layer: one PyTorch-ROCm HIP device or the CPU.

Reference: veles/backends.py:166-948 (``BackendRegistry``, ``Device`` factory,
``AutoDevice``, ``OpenCLDevice``, ``CUDADevice``, ``NumpyDevice``,
``DeviceInfo`` autotuning, device-spec parsing ``"0:0-3x2"``).

The reference's OpenCL / CUDA / NumPy triple collapses into two devices:

* ``HipDevice`` - one MI355X (gfx950).  It owns the compute HIP stream on
  which every unit enqueues its kernels, a communication stream for RCCL
  work, a pinned-host staging pool, and the handle to the hand-written kernel
  library (``veles_amd.ops``).  Per-shape kernel choices (split-K counts)
  come from a per-device JSON table (``devices/gfx950.json``) that the
  autotuner (``veles_amd/ops/autotune.py``) writes - the MI355X analogue of
  the reference ``devices/device_infos.json``.
* ``CpuDevice`` - the reference's "numpy" backend: the same ops evaluated by
  PyTorch on the CPU in float32 (the numerics reference for every kernel).
"""
from __future__ import annotations

import os
import re
import threading

from veles_amd.error import DeviceNotFoundError
from veles_amd.utils.config import root, get
from veles_amd.utils.logger import Logger

__all__ = ["Device", "HipDevice", "CpuDevice", "BackendRegistry",
           "parse_device_spec", "available_backends"]


class BackendRegistry(type):
    backends = {}

    def __init__(cls, name, bases, clsdict):
        super().__init__(name, bases, clsdict)
        backend = clsdict.get("BACKEND")
        if backend:
            BackendRegistry.backends[backend] = cls


def _hip_available():
    try:
        import torch
        return torch.cuda.is_available() and torch.version.hip is not None
    except Exception:
        return False


def available_backends():
    out = ["cpu"]
    if _hip_available():
        out.insert(0, "hip")
    return out


def parse_device_spec(spec):
    """Parse ``"0-3x2"`` / ``"0,2,5"`` / ``"1"`` into a list of device ids
    (``xN`` = N ranks per device, reference backends.py:299-308)."""
    if spec is None or spec == "":
        return [0]
    spec = str(spec)
    if ":" in spec:  # "platform:devices" of the reference; platform ignored
        spec = spec.split(":", 1)[1]
    mult = 1
    m = re.match(r"^(.*)x(\d+)$", spec)
    if m:
        spec, mult = m.group(1), int(m.group(2))
    ids = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            ids.extend(range(int(a), int(b) + 1))
        else:
            ids.append(int(part))
    return [i for i in ids for _ in range(mult)]


class Device(Logger, metaclass=BackendRegistry):
    """Factory: ``Device()`` returns the configured backend's device."""

    BACKEND = None
    PRIORITY = 0

    def __new__(cls, *args, **kwargs):
        if cls is not Device:
            return super().__new__(cls)
        backend = kwargs.pop("backend", None) or get(
            root.common.engine.backend, "auto")
        if backend in ("auto", None):
            backend = "hip" if _hip_available() else "cpu"
        if backend in ("numpy",):
            backend = "cpu"
        if backend in ("ocl", "cuda"):
            raise DeviceNotFoundError(
                "Backend %r does not exist in veles_amd: use 'hip' or 'cpu'" %
                backend)
        klass = BackendRegistry.backends.get(backend)
        if klass is None:
            raise DeviceNotFoundError("Unknown backend %r" % backend)
        inst = super().__new__(klass)
        inst.__init__(*args, **kwargs)
        inst._constructed_by_factory = True
        return inst

    def __init__(self, **kwargs):
        if getattr(self, "_constructed_by_factory", False):
            return
        super().__init__()
        self._lock = threading.Lock()

    # pickling: devices are never pickled with workflows
    def __getstate__(self):
        raise TypeError("Devices are not picklable")

    @property
    def backend_name(self):
        return self.BACKEND

    @property
    def is_gpu(self):
        return False

    @property
    def exists(self):
        return True

    def sync(self):
        pass

    def thread_pool_attach(self, pool):
        pass

    def thread_pool_detach(self, pool):
        pass


class CpuDevice(Device):
    """Reference numerics path (the reference "numpy" backend)."""

    BACKEND = "cpu"
    PRIORITY = 10

    def __init__(self, **kwargs):
        if getattr(self, "_constructed_by_factory", False):
            return
        super().__init__(**kwargs)
        import torch
        self.torch_device = torch.device("cpu")
        self.compute_dtype = torch.float32
        # precision_type "float8" on the CPU simulates the fp8 GEMM inputs
        # (quantize / dequantize) around the float32 reference ops
        self.fp8 = get(root.common.engine.precision_type, "") == "float8"
        self.index = None
        self.device_info = {"name": "cpu", "cores": os.cpu_count()}

    def stream(self):
        return None

    def __repr__(self):
        return "<CpuDevice>"


class HipDevice(Device):
    """One MI355X GPU (one process per GPU; see veles_amd/parallel)."""

    BACKEND = "hip"
    PRIORITY = 30

    def __init__(self, **kwargs):
        if getattr(self, "_constructed_by_factory", False):
            return
        super().__init__(**kwargs)
        import torch
        if not _hip_available():
            raise DeviceNotFoundError("No HIP device is visible")
        idx = kwargs.get("device_id")
        if idx is None:
            idx = get(root.common.engine.device_id, None)
        if idx is None:
            idx = int(os.environ.get("LOCAL_RANK", "0")) % \
                max(1, torch.cuda.device_count())
        self.index = int(idx)
        torch.cuda.set_device(self.index)
        self.torch_device = torch.device("cuda", self.index)
        pt = get(root.common.engine.precision_type, "bfloat16")
        self.compute_dtype = {"float": torch.float32,
                              "float32": torch.float32,
                              "double": torch.float32,
                              "bfloat16": torch.bfloat16,
                              "float16": torch.float16,
                              "float8": torch.bfloat16}.get(
                                  pt, torch.bfloat16)
        self.fp8 = pt == "float8"
        props = torch.cuda.get_device_properties(self.index)
        self.device_info = {
            "name": props.name,
            "gcn_arch": getattr(props, "gcnArchName", ""),
            "cus": props.multi_processor_count,
            "memory_bytes": props.total_memory,
        }
        # The compute stream: every unit kernel, stream-ordered.  RCCL runs
        # the gradient all-reduces on its own internal stream (ordered after
        # this one at each bucket's launch) and the per-bucket updates go to
        # the parameter store's side stream (models/params.py).
        self._compute_stream = torch.cuda.Stream(self.index, priority=0)
        self._pinned_pool = {}
        from veles_amd import ops
        self.ops = ops
        ops.require_library()
        # per-shape kernel choices measured on this device (ops/autotune.py)
        from veles_amd.ops import autotune
        self.tuning = autotune.table()
        self.debug("tuning table %s: %d entries", self.tuning.path,
                   len(self.tuning.entries))

    def stream(self):
        return self._compute_stream

    @property
    def is_gpu(self):
        return True

    def sync(self):
        import torch
        torch.cuda.synchronize(self.index)

    def pinned_buffer(self, nbytes, key=None):
        """Pinned host staging buffer (reused per key)."""
        import torch
        buf = self._pinned_pool.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            if key is not None:
                self._pinned_pool[key] = buf
        return buf

    def max_memory_allocated(self):
        import torch
        return torch.cuda.max_memory_allocated(self.index)

    def __repr__(self):
        return "<HipDevice %d %s>" % (self.index,
                                      self.device_info.get("name"))
