"""Ahead-of-time build of the HIP kernel library ``libhvk.so`` (gfx950).

Every ``csrc/kernels/*.hip`` is compiled with ``hipcc --offload-arch=gfx950``
into an object, then linked into ``veles_amd/ops/libhvk.so`` (in-tree, so it
travels to the GPU box with the repository snapshot).  Objects are cached by
content hash of the source + headers + flags.

Usage: ``python -m veles_amd.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
KDIR = os.path.join(REPO, "csrc", "kernels")
BUILD = os.path.join(REPO, "build", "kernels")
LIB = os.path.join(HERE, "libhvk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HVK_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH,
         "-fgpu-flush-denormals-to-zero", "-munsafe-fp-atomics"]


def _hash(path, extra):
    h = hashlib.sha1()
    with open(path, "rb") as f:
        h.update(f.read())
    for hdr in sorted(glob.glob(os.path.join(KDIR, "*.h"))):
        with open(hdr, "rb") as f:
            h.update(f.read())
    h.update(" ".join(extra).encode())
    return h.hexdigest()[:16]


def _compile(src):
    name = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(BUILD, "%s-%s.o" % (name, _hash(src, FLAGS)))
    if os.path.exists(obj):
        return obj, False
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stderr))
    os.replace(obj + ".tmp", obj)
    return obj, True


def build(force=False, jobs=None, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(KDIR, "*.hip")))
    if not srcs:
        raise RuntimeError("no HIP sources in %s" % KDIR)
    if force:
        for f in glob.glob(os.path.join(BUILD, "*.o")):
            os.remove(f)
    jobs = jobs or min(8, os.cpu_count() or 4, len(srcs))
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(_compile, srcs))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    stamp = hashlib.sha1("".join(sorted(objs)).encode()).hexdigest()
    stamp_file = LIB + ".stamp"
    old = open(stamp_file).read() if os.path.exists(stamp_file) else ""
    if rebuilt or old != stamp or not os.path.exists(LIB):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o",
               LIB + ".tmp"] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stderr)
        os.replace(LIB + ".tmp", LIB)
        with open(stamp_file, "w") as f:
            f.write(stamp)
        if verbose:
            print("built %s from %d sources" % (LIB, len(srcs)))
    elif verbose:
        print("%s is up to date" % LIB)
    return LIB


BENCH_SRC = os.path.join(REPO, "csrc", "bench", "allreduce_bench.cpp")
BENCH_BIN = os.path.join(REPO, "build", "bin", "allreduce_bench")


def build_allreduce_bench(verbose=True):
    """The RCCL all-reduce micro-benchmark (csrc/bench/allreduce_bench.cpp):
    ``build/bin/allreduce_bench [ngpus] [min_mb] [max_mb] [iters] [f32|bf16]``
    (docs/PARALLEL.md).  Rebuilt when the source changes."""
    os.makedirs(os.path.dirname(BENCH_BIN), exist_ok=True)
    stamp = BENCH_BIN + ".stamp"
    h = _hash(BENCH_SRC, ["-lrccl"])
    if os.path.exists(BENCH_BIN) and os.path.exists(stamp) and \
            open(stamp).read() == h:
        return BENCH_BIN
    cmd = [HIPCC, "-O2", "-std=c++17", "--offload-arch=" + ARCH, BENCH_SRC,
           "-o", BENCH_BIN + ".tmp", "-L/opt/rocm/lib", "-lrccl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("allreduce_bench build failed:\n%s" % r.stderr)
    os.replace(BENCH_BIN + ".tmp", BENCH_BIN)
    with open(stamp, "w") as f:
        f.write(h)
    if verbose:
        print("built %s" % BENCH_BIN)
    return BENCH_BIN


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    build(a.force, a.j)
    build_allreduce_bench()


if __name__ == "__main__":
    sys.exit(main())
