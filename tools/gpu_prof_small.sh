#!/bin/bash
# Kernel profiles of the launch-bound small models (batch 100, graphed).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for m in lenet cifar_quick; do
  tools/gpu_step.sh 300 gpurun_out/prof_$m.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$m" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 10 --batch 100 --model $m || exit 1
  grep metric gpurun_out/prof_$m.log
done
