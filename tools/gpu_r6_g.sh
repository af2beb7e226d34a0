#!/bin/bash
# Round 6: conv_hc32 branch-free DMA issue A/B (+ numerics of the variants)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6g}
tools/gpu_step.sh 300 gpurun_out/${T}_pytest.log python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_hc_gpu.py -k "hc32 or forced" || exit 1
tools/gpu_step.sh 400 gpurun_out/${T}_ab.log python3 -u tools/bench_conv_hc_ab.py 2048 5 0 26,27 || exit 1
