#!/bin/bash
# the graph-capture error-drain fix: the test order that failed, then the
# full closing checks
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_order.log python -u -m pytest tests/test_fp8.py tests/test_graphs_gpu.py tests/test_s2d_input.py -m gpu -q --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_order.log
bash tools/gpu_full.sh
