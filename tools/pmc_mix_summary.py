"""Per-kernel instruction mix (pass A) and wave-state shares (pass B) from two
rocprofv3 --pmc counter_collection CSVs (tools/gpu_pmc3.sh), as a markdown
table for profiles/.  Instruction counts are per wave (counter / SQ_WAVES);
MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (time x 2.4 GHz x 1024 SIMDs)."""
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
        key = (n, r["Grid_Size"])
        d = agg.setdefault(key, collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
        d["_ns_" + r["Dispatch_Id"]] = int(r["End_Timestamp"]) - \
            int(r["Start_Timestamp"])
    return agg


def main(a_path, b_path, out, title):
    A, B = load(a_path), load(b_path)
    rows = []
    for k, a in A.items():
        b = B.get(k, {})
        ns = sum(v for kk, v in a.items() if kk.startswith("_ns_"))
        rows.append((ns, k, a, b))
    lines = ["# " + title, "",
             "Per wave: VALU / SALU / VMEM rd / VMEM wr / LDS / MFMA "
             "instructions; wave cycles: wait / issue-stall / active %; "
             "MFMA util % of 1024 SIMDs x 2.4 GHz.", "",
             "| kernel | grid | ms | VALU | SALU | VMEM rd | VMEM wr | LDS | "
             "MFMA | wait % | stall % | active % | MFMA util % |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for ns, k, a, b in sorted(rows, key=lambda x: -x[0])[:30]:
        w = a.get("SQ_WAVES", 0) or 1
        wc = b.get("SQ_WAVE_CYCLES", 0) or 1
        nsb = sum(v for kk, v in b.items() if kk.startswith("_ns_")) or 1
        mf = b.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        lines.append(
            "| %s | %s | %.3f | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f | "
            "%.0f | %.0f | %.0f | %.0f |" % (
                k[0], k[1], ns / 1e6,
                a.get("SQ_INSTS_VALU", 0) / w, a.get("SQ_INSTS_SALU", 0) / w,
                a.get("SQ_INSTS_VMEM_RD", 0) / w,
                a.get("SQ_INSTS_VMEM_WR", 0) / w,
                a.get("SQ_INSTS_LDS", 0) / w,
                a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) / w / 512 * 0 +
                a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) / w,
                100 * b.get("SQ_WAIT_ANY", 0) / wc,
                100 * b.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * b.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                100 * mf / (nsb * 2.4 * 1024)))
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:5])
