#!/bin/bash
# Round 6: halo weight-gradient ablation (no window DMA / no MFMAs)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=r6bb
tools/gpu_step.sh 300 gpurun_out/${T}_abl0.log python3 -u tools/bench_wgrad_ab.py 2048 3 || exit 1
HVK_LIBRARY=build/haloabl/libhvk_halo1.so tools/gpu_step.sh 300 gpurun_out/${T}_abl1.log python3 -u tools/bench_wgrad_ab.py 2048 3 || exit 1
HVK_LIBRARY=build/haloabl/libhvk_halo4.so tools/gpu_step.sh 300 gpurun_out/${T}_abl4.log python3 -u tools/bench_wgrad_ab.py 2048 3 || exit 1
