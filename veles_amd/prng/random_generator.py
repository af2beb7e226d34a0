"""Reproducible keyed random generators.

Reference: veles/prng/random_generator.py:64-295 (a numpy RandomState wrapper
with a keyed global registry ``get(key)``, seed from int / array / file, state
save/restore, thread safety).  Extended with a paired ``torch.Generator`` so
that device-side randomness (dropout masks, weight init on the GPU) is
reproducible from the same seed and is captured in snapshots.
"""
from __future__ import annotations

import os
import threading

import numpy

__all__ = ["RandomGenerator", "get", "xorshift128plus", "xorshift1024star"]


class RandomGenerator(object):
    def __init__(self, key):
        self._key = key
        self._lock = threading.RLock()
        self._rs = numpy.random.RandomState()
        self._seed = None
        self._torch_gen = None

    def __getstate__(self):
        return {"key": self._key, "seed": self._seed, "state": self.state}

    def __setstate__(self, st):
        self.__init__(st["key"])
        self._seed = st["seed"]
        self.state = st["state"]

    @property
    def key(self):
        return self._key

    @property
    def seed_value(self):
        return self._seed

    def seed(self, seed, dtype=None, count=None):
        """Seed from an int, a numpy array, bytes or a file path
        (``file:count[:dtype]`` semantics of the reference CLI)."""
        with self._lock:
            if isinstance(seed, str):
                if os.path.exists(seed):
                    dtype = numpy.dtype(dtype or numpy.uint32)
                    with open(seed, "rb") as f:
                        data = f.read((count or 16) * dtype.itemsize)
                    seed = numpy.frombuffer(data, dtype=dtype)
                else:
                    seed = int(seed, 0)
            if isinstance(seed, bytes):
                seed = numpy.frombuffer(seed, dtype=numpy.uint32)
            if isinstance(seed, numpy.ndarray):
                seed = seed.astype(numpy.uint64).view(numpy.uint32) \
                    if seed.dtype.itemsize == 8 else seed.astype(numpy.uint32)
                self._rs.seed(seed)
                self._seed = seed.tolist()
            else:
                seed = int(seed) & 0xFFFFFFFF
                self._rs.seed(seed)
                self._seed = seed
            self._torch_gen = None

    @property
    def state(self):
        with self._lock:
            st = {"numpy": self._rs.get_state()}
            if self._torch_gen is not None:
                st["torch"] = self._torch_gen.get_state()
            return st

    @state.setter
    def state(self, value):
        with self._lock:
            if isinstance(value, dict):
                self._rs.set_state(value["numpy"])
                if "torch" in value:
                    self.torch_generator().set_state(value["torch"])
            else:
                self._rs.set_state(value)

    def torch_generator(self):
        """A CPU torch.Generator seeded deterministically from this stream."""
        import torch
        if self._torch_gen is None:
            g = torch.Generator()
            g.manual_seed(int(self._rs.randint(0, 2 ** 31 - 1)))
            self._torch_gen = g
        return self._torch_gen

    def __getattr__(self, name):
        # Delegate the numpy.random API (rand, randint, normal, shuffle, ...)
        if name.startswith("_"):
            raise AttributeError(name)
        attr = getattr(self._rs, name)
        if callable(attr):
            def locked(*args, **kwargs):
                with self._lock:
                    return attr(*args, **kwargs)
            return locked
        return attr

    def fill(self, arr, vmin=-1.0, vmax=1.0):
        with self._lock:
            arr[...] = self._rs.uniform(vmin, vmax, arr.shape).astype(
                arr.dtype)

    def fill_normal_real(self, arr, mean, stddev, clip_to_sigma=5.0):
        with self._lock:
            v = self._rs.normal(mean, stddev, arr.shape)
            if clip_to_sigma:
                numpy.clip(v, mean - clip_to_sigma * stddev,
                           mean + clip_to_sigma * stddev, out=v)
            arr[...] = v.astype(arr.dtype)


_generators = {}
_glock = threading.Lock()


def get(key=0):
    """Keyed global generator registry (reference random_generator.py:289)."""
    with _glock:
        g = _generators.get(key)
        if g is None:
            g = RandomGenerator(key)
            g.seed(1234 + (key if isinstance(key, int) else
                           (hash(key) & 0xFFFF)))
            _generators[key] = g
        return g


def all_generators():
    with _glock:
        return dict(_generators)


_MUL1024 = numpy.uint64(1181783497276652981)


def xorshift1024star(states, rounds):
    """numpy model of the device kernel (bit-exact).

    ``states``: uint64 [n_states, 16] (updated in place).  Returns uint64
    [rounds * 16 * n_states] laid out as out[round*16*n + i*n + id]
    (reference ocl/random.cl:42-70).
    """
    states = numpy.asarray(states)
    n = states.shape[0]
    out = numpy.empty(rounds * 16 * n, dtype=numpy.uint64)
    s = states
    with numpy.errstate(over="ignore"):
        for r in range(rounds):
            for i in range(16):
                p = i
                pn = (i + 1) & 15
                s0 = s[:, p].copy()
                s1 = s[:, pn].copy()
                s1 ^= s1 << numpy.uint64(31)
                s1 ^= s1 >> numpy.uint64(11)
                s0 ^= s0 >> numpy.uint64(30)
                s[:, pn] = s0 ^ s1
                out[(r * 16 + i) * n:(r * 16 + i + 1) * n] = s[:, pn] * \
                    _MUL1024
    return out


def xorshift128plus(states, chunk):
    """numpy model of the xorshift128+ kernel: ``states`` uint64 [n, 2];
    thread t generates out[t*chunk + j] from states[t*chunk + j] ... the
    reference indexes one state per output; we follow it exactly
    (reference ocl/random.cl:115-125)."""
    states = numpy.asarray(states)
    out = numpy.empty(states.shape[0], dtype=numpy.uint64)
    with numpy.errstate(over="ignore"):
        s1 = states[:, 0].copy()
        s0 = states[:, 1].copy()
        states[:, 0] = s0
        s1 ^= s1 << numpy.uint64(23)
        states[:, 1] = s1 ^ s0 ^ (s1 >> numpy.uint64(17)) ^ \
            (s0 >> numpy.uint64(26))
        out[:] = states[:, 1] + s0
    return out
