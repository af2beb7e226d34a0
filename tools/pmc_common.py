"""Shared helpers of the rocprofv3 --pmc summary scripts."""
import csv


def load_rows(path, window=False):
    """Rows of a counter_collection CSV; window=True keeps only the
    dispatches strictly between the first and the last hvk_trace_marker
    kernel (bench.py --mark-steps brackets the timed steps with them), so
    the tables hold step kernels only - no dataset generation, warmup or
    library copies."""
    rows = list(csv.DictReader(open(path)))
    if not window:
        return rows
    start = {}
    for r in rows:
        d = r["Dispatch_Id"]
        start.setdefault(d, (int(r["Start_Timestamp"]), r["Kernel_Name"]))
    order = sorted(start.items(), key=lambda kv: kv[1][0])
    marks = [i for i, (_, (_, n)) in enumerate(order)
             if "hvk_trace_marker" in n]
    if len(marks) < 2:
        raise SystemExit("--window: fewer than two trace markers")
    keep = {d for d, _ in order[marks[0] + 1:marks[-1]]}
    return [r for r in rows if r["Dispatch_Id"] in keep]
