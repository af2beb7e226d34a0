#!/bin/bash
# Round 6: conv_hc32 numerics + same-process A/B, resume tests, default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6b}
tools/gpu_step.sh 400 gpurun_out/${T}_pytest.log python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_hc_gpu.py tests/test_resume_gpu.py -s || exit 1
tools/gpu_step.sh 500 gpurun_out/${T}_ab.log python3 -u tools/bench_conv_hc_ab.py 2048 3 256 || exit 1
tools/gpu_step.sh 300 gpurun_out/${T}_bench.log python3 bench.py || exit 1
