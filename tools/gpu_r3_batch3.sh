#!/bin/bash
# GEMM tile variants (96-row wgrad, 48-column dgrad): numerics, e2e, bench,
# step profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/pytest_b3.log python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "gemm or conv or e2e or hip_matches" -m gpu -q -rP --timeout 200 --timeout-method thread || exit 1
grep -E "passed|failed|floor" gpurun_out/pytest_b3.log | tail -6
BATCH=1024 MODEL=alexnet TAG=r3var tools/gpu_prof_step.sh
