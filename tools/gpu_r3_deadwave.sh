#!/bin/bash
# dead-wave MFMA skip in gemm_kernel: numerics (GEMM / conv), A/B rates, bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_deadwave.log python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py tests/test_fp8.py -q -x --timeout 120 --timeout-method thread -k "gemm or conv or wgrad" || exit 1
tail -3 gpurun_out/pytest_deadwave.log
grep -q " passed" gpurun_out/pytest_deadwave.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_deadwave.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_deadwave.log | head -60; exit 1; }
tools/gpu_step.sh 400 gpurun_out/ab_deadwave.log python tools/bench_gemm_ab.py 1024 3 -1 || exit 1
grep -v "^\[" gpurun_out/ab_deadwave.log | head -30
tools/gpu_step.sh 300 gpurun_out/bench_deadwave.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_deadwave.log | cut -c1-200
