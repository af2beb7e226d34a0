#!/bin/bash
# 256-row narrow tiles (gemm_kernel VAR 3 / 4): numerics, A/B (-1 vs 40), bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_tall.log python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pp or gemm or conv or narrow" || exit 1
tail -3 gpurun_out/pytest_tall.log
grep -q " passed" gpurun_out/pytest_tall.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_tall.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_tall.log | head -60; exit 1; }
tools/gpu_step.sh 400 gpurun_out/ab_tall.log python tools/bench_gemm_ab.py 1024 3 -1,40 || exit 1
grep -v "^\[" gpurun_out/ab_tall.log | head -24
tools/gpu_step.sh 300 gpurun_out/bench_tall.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_tall.log | cut -c1-220
