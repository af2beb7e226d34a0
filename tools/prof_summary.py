"""Summarise a rocprofv3 kernel trace CSV into a per-kernel-config table
(markdown) for profiles/."""
import collections
import csv
import sys


def main(trace, out, steps=None, title=""):
    rows = list(csv.DictReader(open(trace)))
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
    lines = ["# %s" % title, "",
             "Total kernel time %.3f ms over %d dispatches." %
             (tot / 1e6, sum(v[0] for v in agg.values())), "",
             "| kernel | grid (x,y,z threads) | VGPR | LDS | calls | "
             "ms/call | total ms | % |", "|---|---|---|---|---|---|---|---|"]
    for k, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        lines.append("| %s | %s,%s,%s | %s | %s | %d | %.3f | %.3f | %.1f |" %
                     (k[0], k[1], k[2], k[3], k[4], k[5], c, d / c / 1e6,
                      d / 1e6, 100.0 * d / tot))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], title=sys.argv[3] if len(sys.argv) > 3
         else "kernel trace")
