#!/bin/bash
# LRN-pool backward: numerics, then AlexNet kernel profiles with the DPP-halo
# kernel off / on (same box, back to back)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_lrn.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lrn or pool" || exit 1
tail -3 gpurun_out/pytest_lrn.log
for v in 0 1 0 1; do
  HVK_LRN_DPP=$v tools/gpu_step.sh 300 gpurun_out/bench_lrn$v.log python bench.py --steps 20 --warmup 5 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_lrn$v.log
done
for v in 0 1; do
  HVK_LRN_DPP=$v tools/gpu_step.sh 300 gpurun_out/prof_lrn$v.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_lrn$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 || exit 1
done
