#!/bin/bash
# ping-pong loop restricted to dense GEMMs + staged split-K atomics: numerics,
# GEMM/conv kernel suite, A/B, bench and a step-only profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_pp2.log python -u -m pytest tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pp or gemm or conv or atomic" || exit 1
tail -3 gpurun_out/pytest_pp2.log
grep -q " passed" gpurun_out/pytest_pp2.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_pp2.log || exit 1
tools/gpu_step.sh 400 gpurun_out/ab_pp2.log python tools/bench_gemm_ab.py 1024 3 -1,32 || exit 1
grep -v "^\[" gpurun_out/ab_pp2.log | head -24
TAG=r3pp2 tools/gpu_prof_step.sh
