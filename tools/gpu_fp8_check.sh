#!/bin/bash
# GPU session: fp8 + GEMM/conv numerics, VGG-16 fp8 / bf16 and AlexNet benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_fp8conv.log python -u -m pytest tests/test_fp8.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fp8 or conv or gemm" || exit 1
tail -2 gpurun_out/pytest_fp8conv.log
grep -q " passed" gpurun_out/pytest_fp8conv.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_fp8conv.log || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_vgg_fp8.log python bench.py --model vgg16 --batch 128 --precision float8 --steps 10 --warmup 3 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_vgg_bf16.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_alex.log python bench.py --steps 20 --warmup 5 || exit 1
grep -h metric gpurun_out/bench_vgg_fp8.log gpurun_out/bench_vgg_bf16.log gpurun_out/bench_alex.log
