#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_fx.log python -u -m pytest tests/test_gemm_fx_gpu.py tests/test_fp8.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_fx.log
tools/gpu_step.sh 300 gpurun_out/bench_device.log python tools/bench_device.py || exit 1
tools/gpu_step.sh 300 gpurun_out/bfp8.log python tools/bench_fp8.py 64 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_fp8.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision float8 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_a.log python bench.py --steps 20 --warmup 5 || exit 1
