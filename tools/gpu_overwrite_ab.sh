#!/bin/bash
# gradient overwrite mode: GPU suite, then AlexNet A/B (off / on)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head
for v in 0 1 0 1; do
  VELES_AMD_GRAD_OVERWRITE=$v tools/gpu_step.sh 300 gpurun_out/bench_ow$v.log python bench.py --steps 20 --warmup 5 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ow$v.log
done
