#!/bin/bash
# rocprofv3 PMC passes (one counter group per run; kernel-trace only) on a
# short AlexNet bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$R/gpurun_out/pmc1" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmc1.log 2>&1
echo "pmc1 rc=$?"
tail -3 gpurun_out/pmc1.log
