#!/bin/bash
# LRN kernels: packed-pair / sliding-sum backward, bare v_exp: numerics,
# micro-benchmark, AlexNet bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_lrn.log python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread -k "lrn or pool or e2e or alexnet" || exit 1
tail -3 gpurun_out/pytest_lrn.log
grep -q " passed" gpurun_out/pytest_lrn.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_lrn.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_lrn.log | head -60; exit 1; }
tools/gpu_step.sh 300 gpurun_out/bench_lrn.log python tools/bench_lrn.py 1024 || exit 1
grep -v "^\[" gpurun_out/bench_lrn.log | tail -12
tools/gpu_step.sh 300 gpurun_out/bench_lrnv.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_lrnv.log | cut -c1-200
