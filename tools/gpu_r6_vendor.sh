#!/bin/bash
# Round 6: resume tests, default bench, MFMA-busy PMC of the conv kernels,
# per-layer bar against MIOpen.  Stops at the first fatal step
# (tools/gpu_step.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/r6_resume_gpu.log python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_resume_gpu.py -s || exit 1
tools/gpu_step.sh 300 gpurun_out/r6_bench_default.log python3 bench.py || exit 1
FILTER="" TAG=r6conv PASSES="A B M" PROBE="tools/bench_conv_vendor.py --probe 2048" \
  tools/gpu_pmc_kernels.sh > gpurun_out/r6_pmc_conv.txt 2>&1 || exit 1
tools/gpu_step.sh 700 gpurun_out/r6_vendor.log python3 -u tools/bench_conv_vendor.py 2048 256 3 || exit 1
