"""Memory-side PMC summary per kernel config from two rocprofv3 --pmc runs
(FETCH_SIZE / TA_BUSY_avr / GRBM_GUI_ACTIVE and WRITE_SIZE / TCC_HIT_sum /
TCC_MISS_sum): HBM read / write bytes and the achieved TB/s over the
kernel's own time, L2 hit rate, texture-address (TA) busy share.
FETCH_SIZE / WRITE_SIZE are in KiB."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_common import load_rows  # noqa: E402

# --window: step kernels only (between the bench's trace markers)
WINDOW = "--window" in sys.argv
if WINDOW:
    sys.argv.remove("--window")


def load(path):
    agg = collections.OrderedDict()
    for r in load_rows(path, WINDOW):
        n = r["Kernel_Name"].replace("void ", "").replace(
            "(anonymous namespace)::", "").split("(")[0][:64]
        d = agg.setdefault((n, r["Grid_Size"]),
                           collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
        d["_ns_" + r["Dispatch_Id"]] = int(r["End_Timestamp"]) - \
            int(r["Start_Timestamp"])
    return agg


def main(p2, p3, out, title):
    a, b = load(p2), load(p3)
    rows = []
    for k, d in a.items():
        ns = sum(v for kk, v in d.items() if kk.startswith("_ns_"))
        e = b.get(k, {})
        rd = d.get("FETCH_SIZE", 0) * 1024
        wr = e.get("WRITE_SIZE", 0) * 1024
        hit, miss = e.get("TCC_HIT_sum", 0), e.get("TCC_MISS_sum", 0)
        gui = d.get("GRBM_GUI_ACTIVE", 0) or 1
        rows.append((ns, k, rd, wr, hit / max(hit + miss, 1),
                     d.get("TA_BUSY_avr", 0) / gui))
    lines = ["# " + title, "",
             "| kernel | grid | ms (sum) | HBM read GB | HBM write GB | "
             "HBM TB/s | L2 hit % | TA busy % |", "|---|---|---|---|---|---|---|---|"]
    for ns, k, rd, wr, hr, ta in sorted(rows, key=lambda x: -x[0])[:25]:
        lines.append("| %s | %s | %.3f | %.3f | %.3f | %.2f | %.0f | %.0f |" % (
            k[0], k[1], ns / 1e6, rd / 1e9, wr / 1e9,
            (rd + wr) / max(ns, 1) / 1e3, 100 * hr, 100 * ta))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:5])
