"""Native inference runtime (the libVeles equivalent) and its bindings.

Reference: libVeles/ (inc/veles/*.h, src/*.cc) — a C++ library that loads a
package written by ``Workflow.package_export`` (contents.json + .npy arrays
in a zip / tar.gz), builds the unit DAG through a name → factory registry,
plans ONE memory arena for every intermediate (MemoryOptimizer,
libVeles/src/memory_optimizer.cc) and runs it.

Here the runtime lives in ``csrc/runtime`` and is compiled by
:func:`build_runtime` into ``veles_amd/runtime/libveles_rt.so`` plus the
``veles_infer`` CLI.  On an MI355X the units run on the same hand-written
gfx950 kernels as training (``libhvk.so``: MFMA GEMM, implicit-GEMM conv,
pooling, LRN, softmax) on bf16 activations inside a device arena; on the CPU
they run float32 reference loops, so a package can be checked anywhere.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os
import subprocess

import numpy

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(REPO, "csrc", "runtime")
LIB = os.path.join(HERE, "libveles_rt.so")
CLI = os.path.join(HERE, "veles_infer")
TEST_BIN = os.path.join(HERE, "veles_rt_tests")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-parameter",
         "-Wno-unused-result"]

__all__ = ["build_runtime", "build_sanitized_tests", "NativeWorkflow",
           "optimize_memory"]


def _sources():
    return sorted(s for s in glob.glob(os.path.join(SRC, "*.cc"))
                  if os.path.basename(s) not in ("veles_infer.cc",
                                                 "tests.cc"))


def _digest(files):
    h = hashlib.sha1()
    for f in sorted(files):
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s failed:\n%s" % (cmd[0], r.stderr[-4000:]))


def build_runtime(force=False, verbose=False):
    """Compile libveles_rt.so, veles_infer and the C++ test binary
    (host code only; GPU work goes through libhvk.so)."""
    from veles_amd.ops import build as kbuild
    if not os.path.exists(kbuild.LIB):
        kbuild.build(verbose=verbose)
    srcs = _sources()
    deps = glob.glob(os.path.join(SRC, "*")) + \
        [os.path.join(REPO, "csrc", "kernels", "hvk_api.h")]
    stamp = _digest(deps)
    stamp_file = LIB + ".stamp"
    if not force and os.path.exists(LIB) and os.path.exists(CLI) and \
            os.path.exists(TEST_BIN) and os.path.exists(stamp_file) and \
            open(stamp_file).read() == stamp:
        return LIB
    opsdir = os.path.dirname(kbuild.LIB)
    link = ["-L" + opsdir, "-lhvk", "-Wl,-rpath,$ORIGIN/../ops",
            "-Wl,-rpath,$ORIGIN", "-lz"]
    _run([HIPCC] + FLAGS + ["-shared", "-o", LIB + ".tmp"] + srcs + link)
    os.replace(LIB + ".tmp", LIB)
    rt_link = ["-L" + HERE, "-lveles_rt"] + link
    _run([HIPCC] + FLAGS + ["-o", CLI, os.path.join(SRC, "veles_infer.cc")]
         + rt_link)
    _run([HIPCC] + FLAGS + ["-o", TEST_BIN, os.path.join(SRC, "tests.cc")]
         + rt_link)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    if verbose:
        print("built", LIB)
    return LIB


SANITIZERS = {"asan": "address,undefined", "tsan": "thread"}


def build_sanitized_tests(kind="asan"):
    """Host-sanitizer build of the C++ self-test binary:
    ``asan`` = AddressSanitizer + UBSan, ``tsan`` = ThreadSanitizer over the
    engine / thread-pool paths.  Host code only (``-fno-gpu-sanitize``):
    GPU ASan / xnack runs are not available on the MI355X pool.  Returns
    the binary path and the environment to run it with."""
    from veles_amd.ops import build as kbuild
    if not os.path.exists(kbuild.LIB):
        kbuild.build()
    out = os.path.join(HERE, "veles_rt_tests_" + kind)
    srcs = sorted(s for s in glob.glob(os.path.join(SRC, "*.cc"))
                  if os.path.basename(s) != "veles_infer.cc")
    stamp = _digest(srcs + glob.glob(os.path.join(SRC, "*.h"))) + kind
    if not (os.path.exists(out) and os.path.exists(out + ".stamp") and
            open(out + ".stamp").read() == stamp):
        opsdir = os.path.dirname(kbuild.LIB)
        _run([HIPCC, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer",
              "-fsanitize=" + SANITIZERS[kind], "-fno-gpu-sanitize",
              "-o", out] + srcs +
             ["-L" + opsdir, "-lhvk", "-Wl,-rpath," + opsdir, "-lz"])
        with open(out + ".stamp", "w") as f:
            f.write(stamp)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:" \
        "abort_on_error=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["TSAN_OPTIONS"] = "halt_on_error=1"
    return out, env


_lib = None


def _load():
    global _lib
    if _lib is None:
        build_runtime()
        lib = ctypes.CDLL(LIB)
        P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
        lib.vr_last_error.restype = ctypes.c_char_p
        lib.vr_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
        lib.vr_free.argtypes = [P]
        lib.vr_free.restype = None
        lib.vr_num_units.argtypes = [P]
        lib.vr_unit_class.argtypes = [P, I]
        lib.vr_unit_class.restype = ctypes.c_char_p
        lib.vr_initialize.argtypes = [P, ctypes.POINTER(L), I, I]
        lib.vr_output_shape.argtypes = [P, ctypes.POINTER(L),
                                        ctypes.POINTER(I)]
        lib.vr_arena_bytes.argtypes = [P]
        lib.vr_arena_bytes.restype = L
        lib.vr_run.argtypes = [P, P, L, P, L]
        lib.vr_set_engine.argtypes = [P, I]
        lib.vr_enable_graph.argtypes = [P, I]
        lib.vr_graph_active.argtypes = [P]
        lib.vr_num_streams.argtypes = [P]
        lib.vr_optimize_memory.argtypes = [ctypes.POINTER(L), I,
                                           ctypes.POINTER(L)]
        lib.vr_optimize_memory.restype = L
        _lib = lib
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(_lib.vr_last_error().decode())


def optimize_memory(nodes):
    """Plan offsets for ``[(start, finish, size), ...]``; returns
    ``(height, positions)`` (libVeles MemoryOptimizer semantics)."""
    lib = _load()
    flat = (ctypes.c_longlong * (3 * len(nodes)))(
        *[int(v) for n in nodes for v in n])
    pos = (ctypes.c_longlong * len(nodes))()
    h = lib.vr_optimize_memory(flat, len(nodes), pos)
    return h, list(pos)


class NativeWorkflow(object):
    """A package loaded into the native runtime."""

    def __init__(self, path):
        lib = _load()
        self._h = ctypes.c_void_p()
        _check(lib.vr_load(os.fsencode(path), ctypes.byref(self._h)))
        self.input_shape = None

    @property
    def unit_classes(self):
        return [_lib.vr_unit_class(self._h, i).decode()
                for i in range(_lib.vr_num_units(self._h))]

    def initialize(self, input_shape, gpu=False):
        shp = (ctypes.c_longlong * len(input_shape))(*input_shape)
        _check(_lib.vr_initialize(self._h, shp, len(input_shape),
                                  1 if gpu else 0))
        self.input_shape = tuple(input_shape)
        out = (ctypes.c_longlong * 8)()
        nd = ctypes.c_int()
        _lib.vr_output_shape(self._h, out, ctypes.byref(nd))
        self.output_shape = tuple(out[i] for i in range(nd.value))

    def set_engine(self, threads=0):
        """threads > 0: run independent branches from a thread pool."""
        _check(_lib.vr_set_engine(self._h, int(threads)))

    def enable_graph(self, on=True):
        """GPU: capture the inference pass into a hipGraph on the 2nd run
        and replay it afterwards."""
        _check(_lib.vr_enable_graph(self._h, 1 if on else 0))

    @property
    def graph_active(self):
        return bool(_lib.vr_graph_active(self._h))

    @property
    def num_streams(self):
        return _lib.vr_num_streams(self._h)

    @property
    def arena_bytes(self):
        return _lib.vr_arena_bytes(self._h)

    def run(self, x):
        x = numpy.ascontiguousarray(x, dtype=numpy.float32)
        if self.input_shape != x.shape:
            self.initialize(x.shape, gpu=getattr(self, "_gpu", False))
        y = numpy.empty(self.output_shape, numpy.float32)
        _check(_lib.vr_run(self._h, x.ctypes.data, x.size, y.ctypes.data,
                           y.size))
        return y

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.vr_free(self._h)
            self._h = None
