#!/bin/bash
# 1-GPU bench + step-only rocprofv3 kernel summary.
# usage: BATCH=1024 MODEL=alexnet TAG=r3 tools/gpu_prof_step.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
B=${BATCH:-1024}; M=${MODEL:-alexnet}; T=${TAG:-r3}; P=${PREC:-bfloat16}
tools/gpu_step.sh 600 gpurun_out/bench_${M}_${T}.log python bench.py --model $M --precision $P --steps 20 --warmup 5 --batch $B || exit 1
tail -2 gpurun_out/bench_${M}_${T}.log
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/prof_${M}_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${M}_${T}" -o run --output-format csv -- python3 "$R/bench.py" --model $M --precision $P --steps 5 --warmup 2 --batch $B --mark-steps || exit 1
f=$(find gpurun_out/prof_${M}_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_${M}_${T}.md "$M b$B 1x MI355X ($P, $T)" --window --steps 5
head -30 gpurun_out/prof_${M}_${T}.md
