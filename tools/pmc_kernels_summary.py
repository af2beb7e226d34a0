"""Summary of tools/gpu_pmc_kernels.sh passes: python3 tools/pmc_kernels_summary.py TAG FILTER"""
import csv, glob, sys, collections
T, filt = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(lambda: collections.defaultdict(int))
ns = collections.defaultdict(list)
for p in "ABFWMLDX":
    f = glob.glob("gpurun_out/pmc_%s_%s/**/*counter_collection.csv" % (T, p), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70] + " grid " + r.get("Grid_Size", r.get("Grid_Size_X", ""))
        if filt not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k][r["Counter_Name"]] += 1
        if p in "BM" and r["Counter_Name"] in ("SQ_WAVE_CYCLES",
                                               "GRBM_GUI_ACTIVE"):
            ns[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, d in agg.items():
    c = calls[k]
    m = {n: d[n] / max(c[n], 1) for n in d}   # per call
    w = max(m.get("SQ_WAVES", 1), 1)
    print(k)
    print("  per wave: VALU %.0f SALU %.0f VMEMrd %.0f VMEMwr %.0f LDS %.0f SMEM %.0f" % tuple(
        m.get(x, 0) / w for x in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SMEM")))
    wc = max(m.get("SQ_WAVE_CYCLES", 1), 1)
    bc = max(m.get("SQ_BUSY_CYCLES", 1), 1)
    print("  wave cycles: wait %.1f%% instwait %.1f%% active %.1f%% valu-active %.1f%% salu-active %.1f%%" % (
        100 * m.get("SQ_WAIT_ANY", 0) / wc, 100 * m.get("SQ_WAIT_INST_ANY", 0) / wc,
        100 * m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * m.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        100 * m.get("SQ_ACTIVE_INST_SCA", 0) / wc))
    if ns[k]:
        ms = sum(ns[k]) / len(ns[k]) / 1e6
        fb, wb = m.get("FETCH_SIZE", 0) * 1024, m.get("WRITE_SIZE", 0) * 1024
        print("  ms/call %.3f  fetch %.1f MB  write %.1f MB  -> %.2f TB/s" % (
            ms, fb / 1e6, wb / 1e6, (fb + wb) / ms / 1e9))
    if "SQ_LDS_IDX_ACTIVE" in m and m.get("GRBM_GUI_ACTIVE"):
        # LDS busy: index-active cycles summed over the CUs (per-SIMD
        # counters sum over 4 SIMDs) against the GPU-active cycles
        act = m["GRBM_GUI_ACTIVE"] / 8.0
        print("  LDS active %.1f%% of CU cycles, bank conflicts %.1f%% of "
              "them, LDS wait %.1f%% of wave cycles" % (
                  100 * m["SQ_LDS_IDX_ACTIVE"] / (act * 256 * 4),
                  100 * m.get("SQ_LDS_BANK_CONFLICT", 0) /
                  max(m["SQ_LDS_IDX_ACTIVE"], 1),
                  100 * m.get("SQ_WAIT_INST_LDS", 0) /
                  max(m.get("SQ_WAVE_CYCLES", 1), 1)))
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
        act = m["GRBM_GUI_ACTIVE"] / 8.0
        print("  MFMA busy %.1f%%, MFMA+VALU co-exec %.1f%% of SIMD cycles; "
              "MFMA / wave %.0f" % (
                  100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (act * 1024),
                  100 * m["SQ_VALU_MFMA_COEXEC_CYCLES"] / (act * 1024),
                  m.get("SQ_INSTS_MFMA", 0) / max(m.get("SQ_WAVES", 1), 1)))
    if "TCC_HIT_sum" in m:
        hit, miss = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
        print("  L2 hit %.1f%%  L1->L2 read requests %.3g  L1 accesses %.3g"
              % (100 * hit / max(hit + miss, 1), m.get(
                  "TCP_TCC_READ_REQ_sum", 0), m.get(
                  "TCP_TOTAL_CACHE_ACCESSES_sum", 0)))
    if m.get("GRBM_GUI_ACTIVE"):
        # MfmaUtil (rocprofiler-sdk counter_defs.yaml): busy cycles summed
        # over the 1024 SIMDs / (max over instances of GPU active cycles x
        # SIMDs).  The csv sums GRBM_GUI_ACTIVE over its 8 XCD instances, so
        # one instance is the sum / 8 (checked: the 1.16 PF conv3 forward
        # reads 48 % = 1.16 / 2.5 PF including its pad-tap MFMAs)
        act = m["GRBM_GUI_ACTIVE"] / 8.0
        print("  MFMA busy %.1f%% of SIMD cycles (CU busy %.1f%%)" % (
            100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (act * 1024),
            100 * m.get("SQ_BUSY_CU_CYCLES", 0) / (act * 256)))
