"""HIP-event timing of the fused LRN -> 3x3/2 max-pool forward / backward on
the AlexNet b1024 shapes (conv1: 55x55x96, conv2: 27x27x256), with the
bytes each moves and the resulting HBM rate."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))

import torch  # noqa: E402

from veles_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    res = {}
    for name, (H, C) in {"conv1": (55, 96), "conv2": (27, 256)}.items():
        x = torch.relu(torch.randn(B, H, H, C, device="cuda")).to(
            torch.bfloat16)
        OH = (H - 3) // 2 + 1
        y = torch.empty(B, OH, OH, C, device="cuda", dtype=torch.bfloat16)
        am = torch.empty(B, OH, OH, C, device="cuda", dtype=torch.uint8)
        dp = torch.randn(B, OH, OH, C, device="cuda").to(torch.bfloat16)
        dx = torch.empty_like(x)
        kw = dict(n=5, alpha=2e-5, beta=0.75, k=1.0)
        f = lambda: ops.lrn_pool_fwd(x, kw["n"], kw["alpha"], kw["beta"],  # noqa
                                     kw["k"], 3, 3, (2, 2), out=y, argmax=am)
        g = lambda: ops.lrn_pool_bwd(x, dp, am, kw["n"], kw["alpha"],  # noqa
                                     kw["beta"], kw["k"], 3, 3, (2, 2),
                                     aux=x, aux_act=3, out=dx)
        setv = getattr(ops._lib.lib(), "hvk_set_lrn_fwd_variant", None)
        tf = None
        if setv is not None:
            # forward A/B (interleaved, median of 5): 0 walk + prefetch with
            # DPP channel halos (the default since round 6), 5 the same walk
            # loading its halos (strips of ~14 rows; 3: ~5, 4: ~9), 1
            # per-output, 2 walk without prefetch; all bit-identical
            vs = (0, 1, 2, 3, 4, 5)
            outs, ts = {}, {v: [] for v in vs}
            for v in vs:
                setv(v)
                f()
                torch.cuda.synchronize()
                outs[v] = (y.clone(), am.clone())
            for _ in range(5):
                for v in vs:
                    setv(v)
                    ts[v].append(timeit(f))
            setv(0)
            same = all(torch.equal(outs[0][0], outs[v][0]) and
                       torch.equal(outs[0][1], outs[v][1]) for v in vs[1:])
            med = {v: sorted(t)[2] for v, t in ts.items()}
            res.setdefault("fwd_ab", {})[name] = {
                "walk_dpp_halo_us": round(med[0], 1), "perout_us": round(med[1], 1),
                "walk_us": round(med[2], 1), "walk_pf_r5_us": round(med[3], 1),
                "walk_pf_r9_us": round(med[4], 1),
                "walk_loaded_halo_us": round(med[5], 1), "bit_identical": same}
            print(name, "fwd DPP-halo walk %.1f us, per-output %.1f us, "
                  "walk %.1f us, strips of 5 %.1f us, of 9 %.1f us, "
                  "loaded-halo walk %.1f us, identical %s" % (
                      med[0], med[1], med[2], med[3], med[4], med[5], same),
                  flush=True)
            tf = med[0]
        setb = getattr(ops._lib.lib(), "hvk_set_lrn_bwd_variant", None)
        tb = None
        if setb is not None:
            # backward A/B: 0 all loads first, 1 loads beside their use
            outs, ts = {}, {0: [], 1: []}
            for v in (0, 1):
                setb(v)
                g()
                torch.cuda.synchronize()
                outs[v] = dx.clone()
            for _ in range(5):
                for v in (0, 1):
                    setb(v)
                    ts[v].append(timeit(g))
            setb(0)
            a, b2 = outs[0].float(), outs[1].float()
            same = bool(torch.equal(outs[0], outs[1]))
            diff = (a != b2) & ~(torch.isnan(a) & torch.isnan(b2))
            nd = int(diff.sum())
            where = None
            if nd:
                idx = diff.nonzero()[0].tolist()
                where = {"first": idx, "a": float(a[tuple(idx)]),
                         "b": float(b2[tuple(idx)])}
            med = {v: sorted(t)[2] for v, t in ts.items()}
            res.setdefault("bwd_ab", {})[name] = {
                "preload_us": round(med[0], 1), "inline_us": round(med[1], 1),
                "bit_identical": same, "n_diff": nd,
                "nan": int(torch.isnan(a).sum()), "first_diff": where}
            print(name, "bwd preload %.1f us, inline %.1f us, identical %s, "
                  "%d differ, %d NaN, %s" % (med[0], med[1], same, nd,
                                            int(torch.isnan(a).sum()), where),
                  flush=True)
            tb = med[0]
        tf, tb = tf or timeit(f), tb or timeit(g)
        bf = x.numel() * 2 + y.numel() * 3
        bb = x.numel() * 4 + dp.numel() * 3
        res[name] = {"fwd_us": round(tf, 1), "fwd_TBps": round(bf / tf / 1e6, 2),
                     "bwd_us": round(tb, 1), "bwd_TBps": round(bb / tb / 1e6, 2)}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
