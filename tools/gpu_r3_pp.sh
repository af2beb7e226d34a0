#!/bin/bash
# ping-pong GEMM loop: numerics (bit-identical to the 128-row loop), A/B on
# the AlexNet / VGG shapes (-1 = ping-pong where eligible, 30 = off), bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_pp.log python -u -m pytest tests/test_gemm_pp_gpu.py -q -x --timeout 120 --timeout-method thread || exit 1
tail -3 gpurun_out/pytest_pp.log
grep -q " passed" gpurun_out/pytest_pp.log && ! grep -q "FAILED\| failed\|rror" gpurun_out/pytest_pp.log || exit 1
tools/gpu_step.sh 400 gpurun_out/ab_pp.log python tools/bench_gemm_ab.py 1024 3 -1,30,32,31 || exit 1
grep -v "^\[" gpurun_out/ab_pp.log | head -24
tools/gpu_step.sh 300 gpurun_out/bench_pp.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_pp.log | cut -c1-220
