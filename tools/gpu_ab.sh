#!/bin/bash
# GPU session: K-loop schedule A/B (kernel bench + AlexNet bench) and the
# weight-gradient split target sweep.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
HVK_GEMM_MODE=1 tools/gpu_step.sh 300 gpurun_out/pytest_oneb.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or gemm" || exit 1
tail -2 gpurun_out/pytest_oneb.log
grep -q " passed" gpurun_out/pytest_oneb.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_oneb.log || exit 1
for m in 0 1; do
  HVK_GEMM_MODE=$m HVK_BENCH_TAG=_m$m tools/gpu_step.sh 300 gpurun_out/bk_m$m.log python tools/bench_kernels.py 512 || exit 1
  HVK_GEMM_MODE=$m tools/gpu_step.sh 300 gpurun_out/bench_m$m.log python bench.py --steps 20 --warmup 5 || exit 1
done
for b in 512 1024 4096; do
  HVK_WGRAD_BLOCKS=$b tools/gpu_step.sh 300 gpurun_out/bench_wg$b.log python bench.py --steps 20 --warmup 5 || exit 1
done
