#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/pytest_all.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tail -2 gpurun_out/pytest_all.log
grep -q " passed" gpurun_out/pytest_all.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_all.log || exit 1
tools/gpu_step.sh 300 gpurun_out/bk96.log python tools/bench_kernels.py 512 || exit 1
tools/gpu_step.sh 300 gpurun_out/bfp8.log python tools/bench_fp8.py 64 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_a.log python bench.py --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_fp8.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision float8 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_bf16.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
