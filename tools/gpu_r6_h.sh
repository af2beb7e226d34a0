#!/bin/bash
# Round 6: conv_hc32 window pitch A/B (Wp = OW + pad)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6h}
tools/gpu_step.sh 500 gpurun_out/${T}_pitch.log python3 -u tools/ab_hc_pitch.py 2048 5 8,2,16 || exit 1
