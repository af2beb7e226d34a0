#!/bin/bash
# 256 x 256 four-phase ping-pong loop: numerics, A/B (-1 = 256x256 where
# eligible, 32 = 256x128 ping-pong, 30 = 128-row loop), bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_pp256.log python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pp or gemm" || exit 1
tail -3 gpurun_out/pytest_pp256.log
grep -q " passed" gpurun_out/pytest_pp256.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_pp256.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_pp256.log | head -60; exit 1; }
tools/gpu_step.sh 400 gpurun_out/ab_pp256.log python tools/bench_gemm_ab.py 1024 3 -1,32,30 || exit 1
grep -v "^\[" gpurun_out/ab_pp256.log | head -8
tools/gpu_step.sh 300 gpurun_out/bench_pp256.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_pp256.log | cut -c1-200
