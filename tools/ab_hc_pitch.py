"""Same-process A/B of the conv_hc window row pitch (hvk_hc_pitch_pad: Wp =
OW + pad) on the AlexNet conv_hc shapes, pads interleaved round by round,
median TF/s.

    python tools/ab_hc_pitch.py [batch] [rounds] [pads, e.g. 8,4,2]"""
import statistics
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from veles_amd.ops import _lib  # noqa: E402
from bench_conv_hc_ab import case, timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    pads = [int(v) for v in sys.argv[3].split(",")] \
        if len(sys.argv) > 3 else [8, 4, 2]
    lib = _lib.lib()
    cases = [("conv2_fwd", ("fwd", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv2_dgrad", ("dgrad", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv3_fwd", ("fwd", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_fwd", ("fwd", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_fwd", ("fwd", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv3_dgrad", ("dgrad", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_dgrad", ("dgrad", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_dgrad", ("dgrad", B, 13, 13, 384, 256, 3, 1, 1, 2))]
    try:
        for name, shp in cases:
            fl, fn = case(*shp)
            res = {p: [] for p in pads}
            for _ in range(rounds):
                for p in pads:
                    lib.hvk_hc_pitch_pad(p)
                    res[p].append(timeit(fn))
            med = {p: statistics.median(v) for p, v in res.items()}
            print("%-12s " % name + "  ".join(
                "pad%d %.1f TF" % (p, fl / med[p] / 1e12) for p in pads),
                flush=True)
    finally:
        lib.hvk_hc_pitch_pad(8)


if __name__ == "__main__":
    main()
