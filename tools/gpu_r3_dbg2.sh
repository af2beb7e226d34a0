#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/pytest_dbg2.log python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -o log_cli=true --log-cli-level=INFO || exit 1
grep -n "HIP error 9\|graphs:\|PASSED\|FAILED" gpurun_out/pytest_dbg2.log | grep -B3 -A1 "graphs:\|HIP error" | tail -60
