#!/bin/bash
# 32x32x16 MFMA A/B: numerics of every GEMM / conv case under the variant,
# then the per-shape interleaved timing against the shipped schedule.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
HVK_TEST_GEMM_VARIANT=2 tools/gpu_step.sh 300 gpurun_out/pytest_mf32.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "conv or gemm" || exit 1
tail -3 gpurun_out/pytest_mf32.log
grep -q " passed" gpurun_out/pytest_mf32.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_mf32.log || exit 1
tools/gpu_step.sh 500 gpurun_out/ab_mf32.log python tools/bench_gemm_ab.py 1024 5 -1,2 || exit 1
cat gpurun_out/ab_mf32.log
