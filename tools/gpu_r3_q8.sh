#!/bin/bash
# fused fp8 output of the bf16 conv epilogues: tests, VGG-16 fp8 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_q8.log python -u -m pytest tests/test_fp8.py tests/test_kernels_gpu.py tests/test_gemm_pp_gpu.py -q -x --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_q8.log
grep -q " passed" gpurun_out/pytest_q8.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_q8.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_q8.log | head -60; exit 1; }
BATCH=128 MODEL=vgg16 PREC=float8 TAG=r3q8 tools/gpu_prof_step.sh
tools/gpu_step.sh 300 gpurun_out/bench_q8_alex.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_q8_alex.log | cut -c1-200
