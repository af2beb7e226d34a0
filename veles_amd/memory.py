"""Host/device mirrored arrays.

Reference: veles/memory.py:110-511 (``Array`` with a numpy ``mem`` and a device
``devmem``; 3-state map protocol; pickling through the host copy;
``shallow_pickle`` minibatch buffers; ``Watcher`` for peak device memory).

Map protocol::

    state 0 = device authoritative, 1 = host copy valid, 2 = host dirty
    map_read:       0 -> D2H copy -> 1
    map_write:      0 -> D2H copy -> 2 ; 1 -> 2
    map_invalidate: 0 -> (sync, no copy) -> 2 ; 1 -> 2
    unmap:          2 -> H2D copy -> 0 ; 1 -> 0

On the CPU device ``devmem`` is a torch view of ``mem`` (zero copy) and all
map calls are free.  On the HIP device ``devmem`` is an HBM tensor whose dtype
may be narrower than the host mirror (bf16 / fp8 on the device, float32 on
the host - numpy has no bf16); copies convert.  Units in the hot loop touch
only ``devmem``; host maps happen for snapshots, metrics and plots.
"""
from __future__ import annotations

import threading

import numpy

__all__ = ["Array", "Watcher", "roundup", "to_numpy_dtype"]


def roundup(num, align):
    d = num % align
    return num if d == 0 else num + (align - d)


def to_numpy_dtype(tdtype):
    import torch
    m = {torch.float32: numpy.float32, torch.float64: numpy.float64,
         torch.float16: numpy.float16, torch.int32: numpy.int32,
         torch.int64: numpy.int64, torch.uint8: numpy.uint8,
         torch.int8: numpy.int8, torch.int16: numpy.int16,
         torch.bool: numpy.bool_, torch.bfloat16: numpy.float32}
    for name in ("float8_e4m3fn", "float8_e5m2"):
        if hasattr(torch, name):
            m[getattr(torch, name)] = numpy.float32
    return m[tdtype]


def _torch_dtype(npdtype):
    import torch
    return {numpy.dtype(numpy.float32): torch.float32,
            numpy.dtype(numpy.float64): torch.float64,
            numpy.dtype(numpy.float16): torch.float16,
            numpy.dtype(numpy.int32): torch.int32,
            numpy.dtype(numpy.int64): torch.int64,
            numpy.dtype(numpy.uint8): torch.uint8,
            numpy.dtype(numpy.int8): torch.int8,
            numpy.dtype(numpy.int16): torch.int16,
            numpy.dtype(numpy.bool_): torch.bool}[numpy.dtype(npdtype)]


class Watcher(object):
    """Tracks device bytes allocated by Arrays (reference memory.py:56-107)."""

    _lock = threading.Lock()
    mem_in_use = 0
    max_mem_in_use = 0

    @staticmethod
    def add(nbytes):
        with Watcher._lock:
            Watcher.mem_in_use += nbytes
            Watcher.max_mem_in_use = max(Watcher.max_mem_in_use,
                                         Watcher.mem_in_use)

    @staticmethod
    def sub(nbytes):
        with Watcher._lock:
            Watcher.mem_in_use -= nbytes


class Array(object):
    """A tensor with a host mirror."""

    def __init__(self, data=None, shallow_pickle=False, device_dtype=None):
        self._mem = None
        self._devmem = None
        self._device = None
        self._state = 1
        self._device_dtype = device_dtype
        self.shallow_pickle = shallow_pickle
        self._shape_hint = None
        self._lock = threading.RLock()
        if data is not None:
            self.reset(data)

    # -- pickling -----------------------------------------------------------
    def __getstate__(self):
        if self.shallow_pickle and self._devmem is not None:
            return {"shallow_pickle": True, "device_dtype": None,
                    "shape": tuple(self._devmem.shape),
                    "dtype": numpy.dtype(to_numpy_dtype(
                        self._devmem.dtype)).str}
        self.map_read()
        st = {"shallow_pickle": self.shallow_pickle,
              "device_dtype": None if self._device_dtype is None
              else str(self._device_dtype)}
        if self.shallow_pickle and self._mem is not None:
            st["shape"] = self._mem.shape
            st["dtype"] = self._mem.dtype.str
        else:
            st["mem"] = self._mem
        return st

    def __setstate__(self, st):
        self.__init__(shallow_pickle=st["shallow_pickle"])
        dd = st.get("device_dtype")
        if dd is not None:
            import torch
            self._device_dtype = getattr(torch, dd.replace("torch.", ""))
        if "mem" in st:
            self._mem = st["mem"]
        elif "shape" in st:
            self._mem = numpy.zeros(st["shape"], dtype=numpy.dtype(st["dtype"]))

    # -- properties ---------------------------------------------------------
    @property
    def mem(self):
        return self._mem

    @mem.setter
    def mem(self, value):
        self.reset(value)

    @property
    def devmem(self):
        return self._devmem

    @devmem.setter
    def devmem(self, tensor):
        """Adopt a device tensor (device becomes authoritative)."""
        with self._lock:
            self._devmem = tensor
            if tensor is not None and tensor.device.type == "cuda":
                self._state = 0
                # host mirror allocated lazily by the first map_*()
                if self._mem is not None and \
                        self._mem.shape != tuple(tensor.shape):
                    self._mem = None
            elif tensor is not None:
                self._mem = tensor.numpy() if tensor.dtype in _NP_OK() \
                    else tensor.float().numpy()
                self._state = 1

    @property
    def device(self):
        return self._device

    @property
    def on_gpu(self):
        return self._devmem is not None and self._devmem.device.type == "cuda"

    def __bool__(self):
        if self._devmem is not None:
            return self._devmem.numel() > 0
        return self._mem is not None and self._mem.size > 0

    def __len__(self):
        sh = self.shape
        return 0 if not sh else sh[0]

    @property
    def shape(self):
        if self._devmem is not None:
            return tuple(self._devmem.shape)
        return None if self._mem is None else self._mem.shape

    @property
    def dtype(self):
        if self._mem is None and self._devmem is not None:
            return numpy.dtype(to_numpy_dtype(self._devmem.dtype))
        return None if self._mem is None else self._mem.dtype

    @property
    def size(self):
        if self._devmem is not None:
            return self._devmem.numel()
        return 0 if self._mem is None else self._mem.size

    @property
    def nbytes(self):
        if self._mem is None and self._devmem is not None:
            return self._devmem.numel() * self._devmem.element_size()
        return 0 if self._mem is None else self._mem.nbytes

    @property
    def sample_size(self):
        return self.size // self.shape[0] if self.size else 0

    def _ensure_host(self):
        if self._mem is None and self._devmem is not None:
            self._mem = numpy.zeros(tuple(self._devmem.shape),
                                    to_numpy_dtype(self._devmem.dtype))

    @property
    def plain(self):
        return self._mem.ravel()

    @property
    def matrix(self):
        return self._mem.reshape(self._mem.shape[0], -1)

    def __getitem__(self, key):
        return self._mem[key]

    def __setitem__(self, key, value):
        self._mem[key] = value

    # -- lifecycle ----------------------------------------------------------
    def reset(self, data=None):
        """Replace the contents (host side); device buffer reallocated lazily
        at the next ``initialize``."""
        with self._lock:
            if self._devmem is not None and self._devmem.device.type == "cuda":
                Watcher.sub(self._devmem.numel() * self._devmem.element_size())
            self._devmem = None
            if data is None:
                self._mem = None
            else:
                import torch
                if isinstance(data, torch.Tensor):
                    data = data.detach().cpu()
                    if data.dtype not in _NP_OK():
                        data = data.float()
                    data = data.numpy()
                self._mem = numpy.ascontiguousarray(data)
            self._state = 1
            dev = self._device
        if dev is not None and self._mem is not None:
            self.initialize(dev)

    def initialize(self, device, device_dtype=None):
        """Allocate / upload the device copy."""
        import torch
        with self._lock:
            self._device = device
            if device_dtype is not None:
                self._device_dtype = device_dtype
            if self._mem is None:
                return
            if device is None or not getattr(device, "is_gpu", False):
                if self._mem.dtype == numpy.float64:
                    pass
                self._devmem = torch.from_numpy(self._mem)
                self._state = 1
                return
            if (self._devmem is not None and
                    tuple(self._devmem.shape) == self._mem.shape and
                    self._devmem.device == device.torch_device):
                if self._state == 2:
                    self.unmap()
                return
            tdt = self._device_dtype or _torch_dtype(self._mem.dtype)
            host = torch.from_numpy(self._mem)
            self._devmem = host.to(device=device.torch_device, dtype=tdt)
            Watcher.add(self._devmem.numel() * self._devmem.element_size())
            self._state = 0

    # -- map protocol -------------------------------------------------------
    @property
    def map_state(self):
        return self._state

    def _d2h(self):
        t = self._devmem
        if t.dtype in _NP_OK() and t.dtype == _torch_dtype(self._mem.dtype):
            self._mem[...] = t.cpu().numpy()
        else:
            self._mem[...] = t.float().cpu().numpy()

    def map_read(self):
        with self._lock:
            self._ensure_host()
            if self._state == 0 and self.on_gpu:
                self._d2h()
                self._state = 1

    def map_write(self):
        with self._lock:
            self._ensure_host()
            if self._state == 0 and self.on_gpu:
                self._d2h()
            if self.on_gpu:
                self._state = 2

    def map_invalidate(self):
        with self._lock:
            self._ensure_host()
            if self._state == 0 and self.on_gpu:
                import torch
                torch.cuda.current_stream(self._devmem.device).synchronize()
            if self.on_gpu:
                self._state = 2

    def unmap(self):
        with self._lock:
            if not self.on_gpu:
                self._state = 1
                return
            if self._state == 2:
                import torch
                host = torch.from_numpy(self._mem)
                self._devmem.copy_(host.to(self._devmem.dtype)
                                   if host.dtype != self._devmem.dtype
                                   else host, non_blocking=False)
            self._state = 0

    # convenience
    def to_numpy(self):
        self.map_read()
        return self._mem

    def __repr__(self):
        return "<Array shape=%s dtype=%s dev=%s state=%d>" % (
            self.shape, self.dtype,
            None if self._devmem is None else self._devmem.dtype,
            self._state)


def _NP_OK():
    import torch
    return (torch.float32, torch.float64, torch.float16, torch.int32,
            torch.int64, torch.uint8, torch.int8, torch.int16, torch.bool)
