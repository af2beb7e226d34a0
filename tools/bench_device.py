"""DeviceBenchmark on the MI355X at the reference's published configuration:
C = A*B, 3001^3, SGEMM and DGEMM at precision levels 0/1/2 (BASELINE.md,
devices/device_infos.json, method veles/backends.py:700-717), plus the bf16
MFMA GEMM.  Writes gpurun_out/bench_device.json."""
import json
import sys

sys.path.insert(0, ".")
from veles_amd.accelerated_units import DeviceBenchmark  # noqa: E402
from veles_amd.backends import Device  # noqa: E402
from veles_amd.dummy import DummyWorkflow  # noqa: E402

# reference seconds per 3001^3 GEMM on a GTX TITAN (device_infos.json)
REF = {("float32", 0): 0.16424, ("float32", 1): 0.17286,
       ("float32", 2): 0.31082, ("float64", 0): 0.33954,
       ("float64", 1): 0.34523, ("float64", 2): 0.70532}

dev = Device(backend="hip")
res = {}
for (dt, lvl), ref_s in REF.items():
    b = DeviceBenchmark(DummyWorkflow(), size=3001, repeats=10, dtype=dt,
                        precision_level=lvl, return_time=True)
    b.initialize(device=dev)
    b.run()
    res["%s_level%d" % (dt, lvl)] = {
        "seconds": b.seconds, "gflops": b.gflops, "ref_seconds": ref_s,
        "ref_gflops": 2 * 3001 ** 3 / ref_s / 1e9,
        "speedup": ref_s / b.seconds}
    print(dt, lvl, res["%s_level%d" % (dt, lvl)], flush=True)
b = DeviceBenchmark(DummyWorkflow(), size=3001, repeats=10, return_time=True)
b.initialize(device=dev)
b.run()
res["bfloat16"] = {"seconds": b.seconds, "gflops": b.gflops}
print("bf16", res["bfloat16"], flush=True)
json.dump(res, open("gpurun_out/bench_device.json", "w"), indent=1)
