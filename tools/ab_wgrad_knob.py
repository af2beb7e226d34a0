"""Same-process A/B of a halo weight-gradient integer knob (an hvk_* setter
taking one int, e.g. hvk_halo_pitch_pad) on the AlexNet layer shapes,
values interleaved round by round, median TF/s.  The knob is left at the
first value.

    python tools/ab_wgrad_knob.py KNOB v0,v1 [batch] [rounds]"""
import statistics
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from veles_amd.ops import _lib  # noqa: E402
from bench_wgrad_ab import timeit  # noqa: E402
import torch  # noqa: E402
import veles_amd.ops as ops  # noqa: E402

BF = torch.bfloat16


def case(N, H, W, C, OC, k, p, g, st=1):
    """bench_wgrad_ab.case that also hands back its dW / dbias"""
    OH, OW = ops.conv_out_size(H, W, k, k, (st, st), (p, p, p, p))
    x = (torch.rand(N, H, W, C, device="cuda") * 2 - 1).to(BF)
    dy = (torch.rand(N, OH, OW, OC, device="cuda") * 2 - 1).to(BF)
    dw = torch.zeros(OC, k, k, C // g, device="cuda")
    db = torch.zeros(OC, device="cuda")
    fl = 2.0 * N * OH * OW * OC * k * k * (C // g)
    return fl, (lambda: ops.conv_wgrad(x, dy, dw, (st, st), (p, p, p, p), g,
                                       dbias=db)), dw, db


def main():
    knob = sys.argv[1]
    vals = [int(v) for v in sys.argv[2].split(",")]
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    setter = getattr(_lib.lib(), knob)
    cases = [("alex_conv2", (B, 27, 27, 96, 256, 5, 2, 2)),
             ("alex_conv3", (B, 13, 13, 256, 384, 3, 1, 1)),
             ("alex_conv4", (B, 13, 13, 384, 384, 3, 1, 2)),
             ("alex_conv5", (B, 13, 13, 384, 256, 3, 1, 2)),
             ("vgg_conv4_2", (B // 8, 28, 28, 512, 512, 3, 1, 1)),
             ("vgg_conv5_2", (B // 8, 14, 14, 512, 512, 3, 1, 1))]
    try:
        for name, shp in cases:
            fl, fn, dw, db = case(*shp)
            got = {}
            for v in vals:   # every setting's result, from zero
                setter(v)
                dw.zero_()
                db.zero_()
                fn()
                torch.cuda.synchronize()
                got[v] = (dw.clone(), db.clone())
            same = all(torch.equal(got[vals[0]][0], got[v][0]) and
                       torch.equal(got[vals[0]][1], got[v][1]) for v in vals)
            res = {v: [] for v in vals}
            for _ in range(rounds):
                for v in vals:
                    setter(v)
                    res[v].append(timeit(fn))
            med = {v: statistics.median(r) for v, r in res.items()}
            print("%-12s " % name + "  ".join(
                "%s=%d %.1f TF" % (knob, v, fl / med[v] / 1e12) for v in vals)
                + "  (%.3fx, bit-identical %s)" % (
                    med[vals[0]] / med[vals[-1]], same), flush=True)
    finally:
        setter(vals[0])


if __name__ == "__main__":
    main()
