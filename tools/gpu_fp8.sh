#!/bin/bash
# GPU session: fp8 kernel tests, fp8 microbench, VGG-16 bf16 vs fp8 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_fp8.log python -u -m pytest tests/test_fp8.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_fp8.log
grep -q " passed" gpurun_out/pytest_fp8.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_fp8.log || exit 1
tools/gpu_step.sh 300 gpurun_out/bfp8.log python tools/bench_fp8.py 64 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_bf16.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_fp8.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision float8 || exit 1
