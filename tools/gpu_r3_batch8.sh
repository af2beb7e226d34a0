#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_b8.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "halo or lrn or conv" || exit 1
tail -2 gpurun_out/pytest_b8.log
grep -q " passed" gpurun_out/pytest_b8.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_b8.log || exit 1
tools/gpu_step.sh 300 gpurun_out/lrn_ab2.log python tools/bench_lrn.py 1024 || exit 1
grep -v "^\[" gpurun_out/lrn_ab2.log | grep -v "^{" | tail -8
BATCH=1024 MODEL=alexnet TAG=r3lrnpre tools/gpu_prof_step.sh
