#!/bin/bash
# Step-only kernel profile of the multi-rank step through a one-rank RCCL
# group with the backward eager (the N > 1 default): where the eager step
# loses against the captured one (GPU busy vs window).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp VELES_AMD_DP_SOLO_COLLECTIVES=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29545
T=${TAG:-solo_eager}
export VELES_AMD_DP_GRAPH_BACKWARD=${GB:-0}
tools/gpu_step.sh 600 gpurun_out/prof_${T}.log rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_${T}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_${T}.md "alexnet b2048 solo RCCL, graph_backward=${GB:-0}" --window --steps 5
rm -rf gpurun_out/prof_${T}
head -4 gpurun_out/prof_${T}.md
