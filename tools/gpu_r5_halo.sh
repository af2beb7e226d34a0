#!/bin/bash
# Round-5 halo wgrad: numerics tests, same-process kernel A/B, then the step
# A/B + profile (tools/gpu_r5_step.sh).  usage: TAG=r5b tools/gpu_r5_halo.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_halo_gpu.py > gpurun_out/halo_test_${T}.log 2>&1 || { tail -30 gpurun_out/halo_test_${T}.log; exit 1; }
tail -3 gpurun_out/halo_test_${T}.log
timeout -k 10 500 python -u tools/bench_wgrad_ab.py 2048 5 256 > gpurun_out/halo_ab_${T}.log 2>&1 || { tail gpurun_out/halo_ab_${T}.log; exit 1; }
cat gpurun_out/halo_ab_${T}.log
[ -n "$STEP" ] && TAG=$T VGG=1 tools/gpu_r5_step.sh
exit 0
