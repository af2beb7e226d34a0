#!/bin/bash
# round-3 closing checks: all-reduce micro-benchmark (1 GPU), full GPU suite,
# smoke, default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 build/bin/allreduce_bench 1 1 256 20 > gpurun_out/allreduce_bench_1gpu.log 2>&1 || exit 1
tail -4 gpurun_out/allreduce_bench_1gpu.log
bash tools/gpu_full.sh
