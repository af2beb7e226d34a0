#!/bin/bash
# fused gather + space-to-depth with dwordx3 source loads: bit-exact tests,
# bench and step-only profile (after the LRN changes)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_s2d2.log python -u -m pytest tests/test_s2d_input.py -q -x --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_s2d2.log
grep -q " passed" gpurun_out/pytest_s2d2.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_s2d2.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_s2d2.log | head -60; exit 1; }
TAG=r3lrnpk tools/gpu_prof_step.sh
