"""Summarise a rocprofv3 kernel trace of tools/probe_branch_overlap.py: the
GEMM kernels per stream, and the time during which GEMMs of two different
streams ran at once (the fan-out branches overlapping).

    python tools/branch_overlap_summary.py TRACE.csv OUT.md"""
import csv
import sys


def main(path, out):
    rows = [r for r in csv.DictReader(open(path))
            if "gemm" in r["Kernel_Name"]]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Stream_Id"], r["Queue_Id"]) for r in rows)
    lines = ["# Fan-out branches on HIP streams: GEMM kernels per stream", "",
             "| stream | queue | GEMM kernels | busy ms |", "|---|---|---|---|"]
    per = {}
    for s, e, st, q in ks:
        d = per.setdefault((st, q), [0, 0])
        d[0] += 1
        d[1] += e - s
    for (st, q), (n, ns) in sorted(per.items()):
        lines.append("| %s | %s | %d | %.3f |" % (st, q, n, ns / 1e6))
    # sweep: time with >= 2 GEMMs of different streams running
    ev = []
    for s, e, st, q in ks:
        ev.append((s, 1, st))
        ev.append((e, -1, st))
    ev.sort()
    live = {}
    both = 0
    last = None
    for t, d, st in ev:
        if last is not None and len([k for k, v in live.items() if v > 0]) >= 2:
            both += t - last
        live[st] = live.get(st, 0) + d
        last = t
    total = (ks[-1][1] - ks[0][0]) if ks else 0
    lines += ["", "GEMM kernels of two different streams running at the same "
              "time: **%.3f ms** of a %.3f ms GEMM span." % (both / 1e6,
                                                           total / 1e6)]
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
