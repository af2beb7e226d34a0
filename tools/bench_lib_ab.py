"""A/B two builds of the GEMM/conv kernels in ONE process (cdna_hip_programming
§5.4 rule 24): the shipped libhvk.so against an experiment build of
gemm.hip (``python tools/bench_lib_ab.py EXP.so [batch] [rounds]``), on the
AlexNet conv shapes with random operands.  Only the GEMM/conv entry points are
swapped, so the experiment library may contain gemm.hip alone."""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
import veles_amd.ops as ops  # noqa: E402
from veles_amd.ops import _lib  # noqa: E402
from bench_gemm_ab import conv, gemm, timeit  # noqa: E402

SWAP = ("hvk_gemm", "hvk_conv_fwd", "hvk_conv_dgrad_t", "hvk_conv_wgrad",
        "hvk_conv_fwd_run", "hvk_conv_wgrad_run", "hvk_im2col")


class Mixed(object):
    def __init__(self, base, exp):
        self._base, self._exp = base, exp

    def __getattr__(self, name):
        return getattr(self._exp if name in SWAP else self._base, name)


def main():
    base = _lib.require_library()
    exp = ctypes.CDLL(sys.argv[1])
    for n in SWAP:
        f = getattr(exp, n)
        f.argtypes = _lib._SIGS[n]
        f.restype = ctypes.c_int
    libs = {"base": base, "exp": Mixed(base, exp)}
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    cases = [("gemm_8192", lambda: gemm(8192, 8192, 8192)),
             ("fc6_fwd", lambda: gemm(B, 4096, 9216)),
             ("fc6_dgrad", lambda: gemm(B, 9216, 4096, tb=False)),
             ("fc6_wgrad", lambda: gemm(4096, 9216, B, ta=True, tb=False)),
             ("fc7_fwd", lambda: gemm(B, 4096, 4096))]
    layers = {"conv1s2d": None,
              "conv2": (B, 27, 27, 96, 256, 5, 1, 2, 2),
              "conv3": (B, 13, 13, 256, 384, 3, 1, 1, 1),
              "conv4": (B, 13, 13, 384, 384, 3, 1, 1, 2),
              "conv5": (B, 13, 13, 384, 256, 3, 1, 1, 2)}
    for name, geo in layers.items():
        if geo is None:
            continue
        for kind in ("fwd", "dgrad", "wgrad"):
            cases.append(("%s_%s" % (name, kind),
                          lambda kind=kind, geo=geo: conv(kind, *geo)))
    for name, make in cases:
        fl, fn = make()
        ts = {k: [] for k in libs}
        for _ in range(rounds):
            for k, lb in libs.items():
                _lib._lib = lb
                ts[k].append(timeit(fn))
        _lib._lib = base
        print(name, " ".join("%s=%.0fTF" % (k, fl / statistics.median(v) /
                                            1e12) for k, v in ts.items()),
              flush=True)
        del fn
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
