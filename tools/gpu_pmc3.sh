#!/bin/bash
# rocprofv3 PMC passes on a short AlexNet bench: counter list, then
# instruction mix (pass A) and wave-state shares (pass B), one pass per run,
# kernel-trace only.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o "SQ_INSTS_[A-Z0-9_]*\|SQ_WAIT[A-Z0-9_]*\|SQ_INST_LEVEL[A-Z0-9_]*\|TCC_EA0_RDREQ[A-Z0-9_]*\|TCC_HIT[a-z_]*\|TCC_MISS[a-z_]*" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_sq.txt || true
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 -d "$R/gpurun_out/pmcA" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmcA.log 2>&1
echo "pmcA rc=$?"
tail -2 gpurun_out/pmcA.log
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$R/gpurun_out/pmcB" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmcB.log 2>&1
echo "pmcB rc=$?"
tail -2 gpurun_out/pmcB.log
