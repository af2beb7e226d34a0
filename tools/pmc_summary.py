"""Summarise a rocprofv3 --pmc counter_collection CSV per kernel config:
wait / issue / active shares of wave cycles, MFMA busy share, LDS bank
conflicts per LDS instruction (MI355X_MICROARCH.md, rocprofv3 PMC slots).

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (kernel time x 2.4 GHz x 1024
SIMDs): the counter sums over every SIMD (calibrated on this box:
SQ_BUSY_CYCLES / (time x 2.4 GHz) = 30 ~ the 32 shader engines).  Under load
the clock can sit below 2.4 GHz, so the figure is a lower bound."""
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


def main(path, out, title):
    rows = list(load_rows(path, WINDOW))
    agg = collections.OrderedDict()
    for r in rows:
        n = r["Kernel_Name"].replace("void ", "").replace(
            "(anonymous namespace)::", "").split("(")[0][:70]
        key = (n, r["Grid_Size"])
        d = agg.setdefault(key, collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
        d["_t"] = max(d["_t"], 0)
        d["_ns_" + r["Dispatch_Id"]] = int(r["End_Timestamp"]) - \
            int(r["Start_Timestamp"])
    lines = ["# " + title, "",
             "| kernel | grid | ms (sum) | wait % | issue-stall % | active % "
             "| MFMA util % (of 1024 SIMDs x 2.4 GHz) | LDS conflict cyc / LDS inst |",
             "|---|---|---|---|---|---|---|---|"]
    items = []
    for k, d in agg.items():
        ns = sum(v for kk, v in d.items() if kk.startswith("_ns_"))
        items.append((ns, k, d))
    for ns, k, d in sorted(items, key=lambda x: -x[0])[:25]:
        wc = d.get("SQ_WAVE_CYCLES", 0) or 1
        lds = d.get("SQ_INSTS_LDS", 0) or 1
        lines.append("| %s | %s | %.3f | %.0f | %.0f | %.0f | %.0f | %.2f |" % (
            k[0], k[1], ns / 1e6, 100 * d.get("SQ_WAIT_ANY", 0) / wc,
            100 * d.get("SQ_WAIT_INST_ANY", 0) / wc,
            100 * d.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            100 * d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(ns * 2.4 * 1024,
                                                             1),
            d.get("SQ_LDS_BANK_CONFLICT", 0) / lds))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
