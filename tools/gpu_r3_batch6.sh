#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_b6.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "lrn" || exit 1
tail -2 gpurun_out/pytest_b6.log
BATCH=1024 MODEL=alexnet TAG=r3walk tools/gpu_prof_step.sh || exit 1
TAG=r3walk tools/gpu_pmc_r3.sh
