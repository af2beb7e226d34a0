"""Summarise a rocprofv3 kernel trace CSV into a per-kernel-config table
(markdown) for profiles/."""
import collections
import csv
import sys


def main(trace, out, steps=None, title="", window=False):
    rows = list(csv.DictReader(open(trace)))
    if window:
        # step-only: the dispatches between the two hvk_trace_marker kernels
        # that bench.py --mark-steps launches around the timed steps
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        idx = [i for i, r in enumerate(rows)
               if "hvk_trace_marker" in r["Kernel_Name"]]
        if len(idx) < 2:
            raise SystemExit("--window: fewer than two trace markers")
        rows = rows[idx[0] + 1:idx[-1]]
        if steps:
            title += " (step-only: %d timed steps between trace markers)" % \
                steps
    agg = collections.OrderedDict()
    for r in rows:
        n = r["Kernel_Name"].replace("void ", "").replace(
            "(anonymous namespace)::", "")
        n = n.split("(")[0][:90]
        key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
               r.get("VGPR_Count", ""), r.get("LDS_Block_Size", ""))
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(key, [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    busy = ""
    if window and rows:
        # the union of the dispatch intervals (concurrent streams overlap):
        # what is left of the window is GPU idle time
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                    for r in rows)
        u, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                u, cs, ce = u + ce - cs, s, e
            else:
                ce = max(ce, e)
        u += ce - cs
        span = iv[-1][1] - iv[0][0]
        busy = (" Busy (union of dispatches) %.3f ms of a %.3f ms window"
                "%s; idle %.3f ms." % (u / 1e6, span / 1e6,
                                       (" (%.3f / %.3f ms per step)" % (
                                           u / 1e6 / steps, span / 1e6 / steps))
                                       if steps else "", (span - u) / 1e6))
    lines = ["# %s" % title, "",
             "Total kernel time %.3f ms over %d dispatches%s." %
             (tot / 1e6, sum(v[0] for v in agg.values()),
              ("; %.3f ms of kernel time per step" % (tot / 1e6 / steps))
              if steps else "") + busy, "",
             "| kernel | grid (x,y,z threads) | VGPR | LDS | calls | "
             "ms/call | total ms | ms/step | % |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        lines.append("| %s | %s,%s,%s | %s | %s | %d | %.3f | %.3f | %s | %.1f |"
                     % (k[0], k[1], k[2], k[3], k[4], k[5], c, d / c / 1e6,
                        d / 1e6, ("%.3f" % (d / 1e6 / steps)) if steps
                        else "-", 100.0 * d / tot))
    if window and steps and len(rows) % steps == 0:
        # the last timed step in dispatch order (which layer is which kernel)
        per = len(rows) // steps
        lines += ["", "## Last timed step in dispatch order", "",
                  "| # | kernel | grid x | ms |", "|---|---|---|---|"]
        for i, r in enumerate(rows[-per:]):
            n = r["Kernel_Name"].replace("void ", "").replace(
                "(anonymous namespace)::", "").split("(")[0][:90]
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            lines.append("| %d | %s | %s | %.3f |" % (i, n, r["Grid_Size_X"],
                                                      d / 1e6))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("title", nargs="?", default="kernel trace")
    ap.add_argument("--window", action="store_true",
                    help="keep only dispatches between the trace markers")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps inside the window (per-step column)")
    a = ap.parse_args()
    main(a.trace, a.out, steps=a.steps, title=a.title, window=a.window)
