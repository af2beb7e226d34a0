#!/bin/bash
# LDS-halo conv kernels: numerics vs the implicit GEMM, A/B timing; then the
# step profile and PMC passes of the resulting build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_b7.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "halo or lrn or conv" || exit 1
tail -3 gpurun_out/pytest_b7.log
grep -q " passed" gpurun_out/pytest_b7.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_b7.log || exit 1
tools/gpu_step.sh 400 gpurun_out/halo_ab.log python tools/bench_halo_ab.py 1024 5 || exit 1
grep -v "^\[" gpurun_out/halo_ab.log | grep -v "^{" | tail -12
BATCH=1024 MODEL=alexnet TAG=r3halo tools/gpu_prof_step.sh || exit 1
TAG=r3halo tools/gpu_pmc_r3.sh
