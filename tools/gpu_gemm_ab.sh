#!/bin/bash
# GPU session: GEMM/conv numerics, in-process A/B of the shipped kernels
# against an older build of gemm.hip (${AB_LIB:-veles_amd/ops/libhvk_gemmprev.so}),
# then the AlexNet bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_gemmconv.log python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or gemm or fp8" || exit 1
tail -2 gpurun_out/pytest_gemmconv.log
grep -q " passed" gpurun_out/pytest_gemmconv.log && ! grep -q "FAILED\| failed\|rror" gpurun_out/pytest_gemmconv.log || exit 1
tools/gpu_step.sh 300 gpurun_out/ab_gemm.log python tools/bench_lib_ab.py ${AB_LIB:-veles_amd/ops/libhvk_gemmprev.so} 512 5 || exit 1
cat gpurun_out/ab_gemm.log
tools/gpu_step.sh 300 gpurun_out/bench_ab.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_ab.log
