#!/bin/bash
# GPU session: big-tile GEMM correctness + A/B kernel bench + AlexNet bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_big.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "big_tile or conv or gemm" || exit 1
tail -3 gpurun_out/pytest_big.log
grep -q " passed" gpurun_out/pytest_big.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_big.log || exit 1
HVK_BIG_TILE=0 tools/gpu_step.sh 300 gpurun_out/bk0.log python tools/bench_kernels.py 512 || exit 1
HVK_BIG_TILE=1 tools/gpu_step.sh 300 gpurun_out/bk1.log python tools/bench_kernels.py 512 || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_big.log python bench.py --steps 20 --warmup 5 || exit 1
