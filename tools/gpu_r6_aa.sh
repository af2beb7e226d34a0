#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6aa
tools/gpu_step.sh 300 gpurun_out/${T}_test.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_hc_gpu.py tests/test_alexnet_bench_scale_gpu.py || exit 1
tools/gpu_step.sh 500 gpurun_out/${T}_ab.log python3 -u tools/ab_hc_lib.py build/ab/libhvk_hc_pre24.so 2048 5 || exit 1
EXP=build/ab/libhvk_hc_pre24.so TAG=${T}b ROUNDS=2 bash tools/gpu_bench_ab.sh || exit 1
