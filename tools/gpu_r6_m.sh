#!/bin/bash
# Round 6: lean conv_hc32 loop - numerics, then the epilogue ablation
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6m}
tools/gpu_step.sh 300 gpurun_out/${T}_test.log python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_hc_gpu.py || exit 1
HVK_LIBRARY=build/hcabl/libhvk_hcabl.so tools/gpu_step.sh 400 gpurun_out/${T}_abl.log python3 -u tools/ablate_conv_hc.py 2048 5 0,32,64,1 || exit 1
