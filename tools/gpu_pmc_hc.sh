#!/bin/bash
# PMC passes over tools/probe_conv_hc.py (conv_hc and the implicit GEMM).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-probe}
for pass in A B L; do
  case $pass in
    A) ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16" ;;
    B) ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" ;;
    L) ctr="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE" ;;
  esac
  tools/gpu_step.sh 200 gpurun_out/pmc_${T}_$pass.log timeout -s KILL 150 \
    rocprofv3 --kernel-trace --pmc $ctr -d "$R/gpurun_out/pmc_${T}_$pass" \
    -o run --output-format csv -- python3 "$R/tools/probe_conv_hc.py" 2048 || exit 1
done
python3 - "$T" <<'PY'
import csv, glob, sys, collections
T = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
ns = collections.defaultdict(list)
for p in "ABL":
    f = glob.glob("gpurun_out/pmc_%s_%s/**/*counter_collection.csv" % (T, p), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if p == "B":
            ns[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, d in agg.items():
    if "conv_hc" not in k and "gemm" not in k:
        continue
    w = max(d.get("SQ_WAVES", 1), 1)
    print(k)
    print("  per wave: VALU %.0f SALU %.0f VMEMrd %.0f VMEMwr %.0f LDS %.0f MFMA %.0f" % tuple(
        d.get(c, 0) / w for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_VALU_MFMA_MOPS_BF16")))
    wc = max(d.get("SQ_WAVE_CYCLES", 1), 1)
    print("  wait %.1f%% instwait %.1f%% active %.1f%% lds-instwait %.1f%%  mfma busy/busy %.2f  lds conflicts/idx %.3f" % (
        100 * d.get("SQ_WAIT_ANY", 0) / wc, 100 * d.get("SQ_WAIT_INST_ANY", 0) / wc,
        100 * d.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * d.get("SQ_WAIT_INST_LDS", 0) / wc,
        d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(d.get("SQ_BUSY_CYCLES", 1), 1),
        d.get("SQ_LDS_BANK_CONFLICT", 0) / max(d.get("SQ_LDS_IDX_ACTIVE", 1), 1)))
    if ns[k]:
        print("  ms/call %.3f" % (sum(ns[k]) / len(ns[k]) / 1e6))
PY
exit 0
