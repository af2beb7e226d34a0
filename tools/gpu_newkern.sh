#!/bin/bash
# numerics of the xact / gather / stochastic-pool kernels + graphed workflows
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_newkern.log python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k "xact or gather or stochastic or depool or graph" || exit 1
tail -30 gpurun_out/pytest_newkern.log
