#!/bin/bash
# GPU session: 128-vs-64 tile threshold A/B (HVK_BN_WASTE_DIV) on the
# AlexNet step and the per-layer kernel bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_gemm.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or conv" || exit 1
tail -1 gpurun_out/pytest_gemm.log
for d in 8 2 1; do
  HVK_BN_WASTE_DIV=$d tools/gpu_step.sh 300 gpurun_out/bench_bn$d.log python bench.py --steps 20 --warmup 5 || exit 1
  HVK_BN_WASTE_DIV=$d tools/gpu_step.sh 300 gpurun_out/bk_bn$d.log python tools/bench_kernels.py 512 || exit 1
done
for d in 8 2; do
  HVK_BN_WASTE_DIV=$d tools/gpu_step.sh 300 gpurun_out/vgg_bn$d.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
done
