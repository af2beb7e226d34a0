#!/bin/bash
# s2d / fill kernels: numerics, then AlexNet kernel profile with the row
# kernel off / on
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_s2d.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "space_to_depth or conv or fill or minibatch" || exit 1
tail -3 gpurun_out/pytest_s2d.log
for v in 0 1; do
  HVK_S2D_ROWS=$v tools/gpu_step.sh 300 gpurun_out/prof_s2d$v.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_s2d$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 || exit 1
done
for v in 0 1 0 1; do
  HVK_S2D_ROWS=$v tools/gpu_step.sh 300 gpurun_out/bench_s2d$v.log python bench.py --steps 20 --warmup 5 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_s2d$v.log
done
