#!/bin/bash
# GPU session: whole GPU suite, then the row-marching LRN-pool forward A/B
# (HVK_LRN_FWD_ROWS=0 / 1) on the AlexNet bench, then a kernel profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} || exit 1
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
for v in 0 1 0 1; do
  HVK_LRN_FWD_ROWS=$v tools/gpu_step.sh 300 gpurun_out/bench_rows$v.log python bench.py --steps 20 --warmup 5 || exit 1
  grep -h metric gpurun_out/bench_rows$v.log | cut -c1-160
done
tools/gpu_step.sh 600 gpurun_out/prof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 || exit 1
grep metric gpurun_out/prof.log | cut -c1-160
