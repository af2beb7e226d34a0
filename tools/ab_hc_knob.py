"""Same-process A/B of a conv_hc integer knob (an hvk_* setter taking one
int, e.g. hvk_hc32_ts or hvk_hc_pitch_pad) on the AlexNet conv_hc shapes,
values interleaved round by round, median TF/s.  The knob is left at the
first value.

    python tools/ab_hc_knob.py KNOB v0,v1[,...] [batch] [rounds]"""
import statistics
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from veles_amd.ops import _lib  # noqa: E402
from bench_conv_hc_ab import case, timeit  # noqa: E402


def main():
    knob = sys.argv[1]
    vals = [int(v) for v in sys.argv[2].split(",")]
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    setter = getattr(_lib.lib(), knob)
    cases = [("conv1_fwd", ("fwd", B, 227, 227, 3, 96, 11, 4, 0, 1)),
             ("conv3_fwd", ("fwd", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_fwd", ("fwd", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_fwd", ("fwd", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv3_dgrad", ("dgrad", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_dgrad", ("dgrad", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_dgrad", ("dgrad", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("vgg_conv4_2_fwd", ("fwd", B // 4, 28, 28, 512, 512, 3, 1, 1,
                                  1)),
             ("vgg_conv3_2_dgrad", ("dgrad", B // 4, 56, 56, 256, 256, 3, 1,
                                    1, 1))]
    try:
        for name, shp in cases:
            fl, fn = case(*shp)
            res = {v: [] for v in vals}
            for _ in range(rounds):
                for v in vals:
                    setter(v)
                    res[v].append(timeit(fn))
            med = {v: statistics.median(r) for v, r in res.items()}
            print("%-18s " % name + "  ".join(
                "%s=%d %.1f TF" % (knob, v, fl / med[v] / 1e12) for v in vals)
                + "  (%.3fx)" % (med[vals[0]] / med[vals[-1]]), flush=True)
    finally:
        setter(vals[0])


if __name__ == "__main__":
    main()
