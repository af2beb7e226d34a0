#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_r3_batch8.sh || exit 1
# GEMM main-loop ablation (diagnostic variants, wrong results by design):
# -1 shipped, 11 half the MFMAs, 12 no DMA after the first K tile, 13 no DMA
# and no barriers after it
tools/gpu_step.sh 500 gpurun_out/ab_ablation.log python tools/bench_gemm_ab.py 1024 3 -1,11,12,13 || exit 1
grep -v "^\[" gpurun_out/ab_ablation.log | head -12
