#!/bin/bash
# GPU session: GPU test suite, then smoke + bench + kernel bench + rocprofv3 stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_gpu.log
BATCH=${BATCH:-512} bash tools/gpu_bench_prof.sh
