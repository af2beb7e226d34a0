#!/bin/bash
# Round 6: conv_hc32 packed-bf16 ReLU epilogues - numerics, A/B vs HEAD build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6o}
tools/gpu_step.sh 300 gpurun_out/${T}_test.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_hc_gpu.py tests/test_alexnet_bench_scale_gpu.py || exit 1
tools/gpu_step.sh 500 gpurun_out/${T}_ab.log python3 -u tools/ab_hc_lib.py build/ab/libhvk_hc_head.so 2048 7 || exit 1
