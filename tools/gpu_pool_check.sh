#!/bin/bash
# GPU session: pooling / LRN numerics, then AlexNet and VGG-16 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_pool.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or lrn" || exit 1
tail -2 gpurun_out/pytest_pool.log
grep -q " passed" gpurun_out/pytest_pool.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_pool.log || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_alex.log python bench.py --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_vgg_bf16.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
grep -h metric gpurun_out/bench_alex.log gpurun_out/bench_vgg_bf16.log
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/prof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 || exit 1
