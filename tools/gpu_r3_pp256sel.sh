#!/bin/bash
# round-aware 256x256 selection: numerics, A/B (-1 = new rule, 32 = 256x128), bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_pp256sel.log python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pp or gemm or fc or all2all" || exit 1
tail -2 gpurun_out/pytest_pp256sel.log
grep -q " passed" gpurun_out/pytest_pp256sel.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_pp256sel.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_pp256sel.log | head -60; exit 1; }
tools/gpu_step.sh 400 gpurun_out/ab_pp256sel.log python tools/bench_gemm_ab.py 1024 5 -1,32 || exit 1
grep -v "^\[" gpurun_out/ab_pp256sel.log | head -7
tools/gpu_step.sh 300 gpurun_out/bench_pp256sel.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_pp256sel.log | cut -c1-170
