#!/bin/bash
# the round-end checks: whole GPU suite, smoke(), default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 gpurun_out/smoke.log
tools/gpu_step.sh 300 gpurun_out/bench_default.log python bench.py || exit 1
grep metric gpurun_out/bench_default.log
