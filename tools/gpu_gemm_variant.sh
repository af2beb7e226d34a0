#!/bin/bash
# GPU session: GEMM variant 1 (HVK_GEMM_VARIANT) numerics + A/B vs the shipped loop.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
HVK_GEMM_VARIANT=1 tools/gpu_step.sh 300 gpurun_out/pytest_var.log python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_fx_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or gemm" || exit 1
tail -2 gpurun_out/pytest_var.log
grep -q " passed" gpurun_out/pytest_var.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_var.log || exit 1
tools/gpu_step.sh 400 gpurun_out/ab_var.log python tools/bench_gemm_ab.py 512 5 0,1 || exit 1
for v in 0 1; do
  HVK_GEMM_VARIANT=$v tools/gpu_step.sh 300 gpurun_out/bench_var_v$v.log python bench.py --steps 20 --warmup 5 || exit 1
done
grep metric gpurun_out/bench_var_v*.log
