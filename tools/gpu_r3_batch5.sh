#!/bin/bash
# single-rank overlapped update: graph + numerics tests, bench, step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/pytest_b5.log python -u -m pytest tests/test_graphs_gpu.py tests/test_kernels_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "graph or overlap or gemm or conv" || exit 1
tail -3 gpurun_out/pytest_b5.log
grep -q " passed" gpurun_out/pytest_b5.log && ! grep -q "FAILED\| failed\|rror" gpurun_out/pytest_b5.log || exit 1
BATCH=1024 MODEL=alexnet TAG=r3ovl tools/gpu_prof_step.sh
