#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_native_asan.sh || exit 1
tools/gpu_step.sh 400 gpurun_out/pytest_b1.log python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_native_runtime.py -k "lrn or e2e or hip_matches or native" -m gpu -v --timeout 200 --timeout-method thread || exit 1
grep -E "passed|failed" gpurun_out/pytest_b1.log | tail -3
tools/gpu_step.sh 300 gpurun_out/fc_ab.log python tools/bench_fc_ab.py 1024 5 || exit 1
tail -12 gpurun_out/fc_ab.log
BATCH=1024 TAG=r3lrn4 tools/gpu_prof_step.sh
