#!/bin/bash
# fp8 weight gradient: numerics, VGG-16 fp8 b128 bench + step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_fp8w.log python -u -m pytest tests/test_fp8.py -v -x --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_fp8w.log
grep -q " passed" gpurun_out/pytest_fp8w.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_fp8w.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_fp8w.log | head -60; exit 1; }
BATCH=128 MODEL=vgg16 PREC=float8 TAG=r3fp8w tools/gpu_prof_step.sh
tools/gpu_step.sh 400 gpurun_out/bench_vgg_bf16.log python bench.py --model vgg16 --precision bfloat16 --steps 20 --warmup 5 --batch 128 || exit 1
grep metric gpurun_out/bench_vgg_bf16.log | cut -c1-200
