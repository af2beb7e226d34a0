#!/bin/bash
# fused gather + space-to-depth with all loads first: bit-exact tests, step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_s2d.log python -u -m pytest tests/test_s2d_input.py tests/test_e2e_gpu.py -q -x --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_s2d.log
grep -q " passed" gpurun_out/pytest_s2d.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_s2d.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_s2d.log | head -60; exit 1; }
TAG=r3s2d tools/gpu_prof_step.sh
