#!/bin/bash
# which GPU test leaves a HIP error pending (HVK_DEBUG_LAST_ERROR=1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
HVK_DEBUG_LAST_ERROR=1 tools/gpu_step.sh 600 gpurun_out/pytest_dbg.log python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -o log_cli=true --log-cli-level=WARNING || exit 1
grep -n "pending HIP error" gpurun_out/pytest_dbg.log | head -20
tail -3 gpurun_out/pytest_dbg.log
grep -n "capture\|WARNING" gpurun_out/pytest_dbg.log | tail -30
tools/gpu_step.sh 300 gpurun_out/bench_dbg.log python bench.py --steps 20 --warmup 5 || exit 1
grep -i "metric\|ran while the capture" gpurun_out/bench_dbg.log | cut -c1-200
