#!/bin/bash
# rocprofv3 PMC passes on the AlexNet b1024 bench (2 timed steps): the
# instruction mix (A), wave states (B), HBM read + TA busy (C), HBM write +
# L2 hit rate (D) - one counter set per run, kernel trace only - and their
# per-kernel summaries.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r3}
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d "$R/gpurun_out/pmc_$n" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmc_$n.log 2>&1
  local rc=$?
  echo "pmc $n rc=$rc"
  return $rc
}
run A SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 || exit 1
run B SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run C FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE || exit 1
run D WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit 1
fa=$(find gpurun_out/pmc_A -name "*counter_collection.csv" | head -1)
fb=$(find gpurun_out/pmc_B -name "*counter_collection.csv" | head -1)
fc=$(find gpurun_out/pmc_C -name "*counter_collection.csv" | head -1)
fd=$(find gpurun_out/pmc_D -name "*counter_collection.csv" | head -1)
python tools/pmc_mix_summary.py "$fa" "$fb" gpurun_out/pmc_mix_$T.md "AlexNet b1024 1x MI355X: instruction mix and wave states ($T)"
python tools/pmc_mem_summary.py "$fc" "$fd" gpurun_out/pmc_mem_$T.md "AlexNet b1024 1x MI355X: HBM traffic, L2 hit rate, TA busy ($T)"
head -30 gpurun_out/pmc_mix_$T.md
head -30 gpurun_out/pmc_mem_$T.md
