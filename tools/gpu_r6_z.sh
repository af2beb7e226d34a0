#!/bin/bash
# Round 6: staged epilogue stores on backward-data only - numerics and
# whole-step A/B against the previous conv_hc build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6z}
tools/gpu_step.sh 300 gpurun_out/${T}_test.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_hc_gpu.py || exit 1
EXP=build/ab/libhvk_hc_prets.so TAG=${T}b ROUNDS=3 bash tools/gpu_bench_ab.sh || exit 1
