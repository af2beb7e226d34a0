#!/bin/bash
# GPU session: rocprofv3 kernel stats of a short AlexNet bench run.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B=${BATCH:-512}
MODEL=${MODEL:-alexnet}
tools/gpu_step.sh 600 gpurun_out/prof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --batch $B --model $MODEL || exit 1
grep metric gpurun_out/prof.log
