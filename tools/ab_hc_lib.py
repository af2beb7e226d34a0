"""Same-process A/B of two builds of the halo conv kernels (conv_hc.hip):
the shipped libhvk.so against an experiment build (tools/build_ab_lib.py
conv_hc REV OUT.so, e.g. the previous commit's source), on the AlexNet
conv_hc shapes with random operands; only the conv_hc entry points are
swapped, builds interleaved round by round (cdna_hip_programming.md §5.4
rule 24), median TF/s.

    python tools/ab_hc_lib.py EXP.so [batch] [rounds]"""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from veles_amd.ops import _lib  # noqa: E402
from bench_conv_hc_ab import case, timeit  # noqa: E402

SWAP = ("hvk_conv_fwd_hc", "hvk_conv_dgrad_hc", "hvk_conv_hc_wpack_bytes",
        "hvk_hc_variant", "hvk_hc32", "hvk_hc_last_variant",
        "hvk_hc_pitch_pad")


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
        f.restype = ctypes.c_longlong if n in _lib._LL_RET else ctypes.c_int
    libs = {"new": base, "exp": Mixed(base, exp)}
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    cases = [("conv3_fwd", ("fwd", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_fwd", ("fwd", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_fwd", ("fwd", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv3_dgrad", ("dgrad", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_dgrad", ("dgrad", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_dgrad", ("dgrad", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv1_fwd", ("fwd", B, 227, 227, 3, 96, 11, 4, 0, 1)),
             ("conv2_fwd", ("fwd", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv2_dgrad", ("dgrad", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("vgg_conv4_2_fwd", ("fwd", B // 4, 28, 28, 512, 512, 3, 1, 1,
                                  1)),
             ("vgg_conv3_2_dgrad", ("dgrad", B // 4, 56, 56, 256, 256, 3, 1,
                                    1, 1))]
    try:
        for name, shp in cases:
            fl, fn = case(*shp)
            ts = {k: [] for k in libs}
            for _ in range(rounds):
                for k, lb in libs.items():
                    _lib._lib = lb
                    ts[k].append(timeit(fn))
            med = {k: statistics.median(v) for k, v in ts.items()}
            print("%-18s " % name + "  ".join(
                "%s %.1f TF" % (k, fl / med[k] / 1e12) for k in libs) +
                "  (new/exp %.3fx)" % (med["exp"] / med["new"]), flush=True)
            del fn
            torch.cuda.empty_cache()
    finally:
        _lib._lib = base


if __name__ == "__main__":
    main()
