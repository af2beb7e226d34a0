#!/bin/bash
# Round 6: bench-scale gate, N>1 path through a one-rank RCCL group at
# b3072 (eager vs captured backward) against dp1, LDS / co-exec PMC of conv_hc32
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6d}
tools/gpu_step.sh 500 gpurun_out/${T}_pytest.log python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_alexnet_bench_scale_gpu.py tests/test_conv_hc_gpu.py -s || exit 1
for i in 1 2; do
  tools/gpu_step.sh 300 gpurun_out/${T}_dp1_$i.log python3 bench.py || exit 1
  VELES_AMD_DP_SOLO_COLLECTIVES=1 VELES_AMD_DP_GRAPH_BACKWARD=0 tools/gpu_step.sh 300 gpurun_out/${T}_solo_eager_$i.log python3 bench.py || exit 1
  VELES_AMD_DP_SOLO_COLLECTIVES=1 VELES_AMD_DP_GRAPH_BACKWARD=0 VELES_AMD_WGRAD_STREAM=1 tools/gpu_step.sh 300 gpurun_out/${T}_solo_eager_side_$i.log python3 bench.py || exit 1
  VELES_AMD_DP_SOLO_COLLECTIVES=1 tools/gpu_step.sh 300 gpurun_out/${T}_solo_graph_$i.log python3 bench.py || exit 1
  VELES_AMD_DP_SOLO_COLLECTIVES=1 VELES_AMD_DP_GRAPH_BACKWARD=validate tools/gpu_step.sh 300 gpurun_out/${T}_solo_validate_$i.log python3 bench.py || exit 1
done
tools/gpu_step.sh 400 gpurun_out/${T}_ab_opt.log python3 -u tools/bench_conv_hc_ab.py 2048 3 0 26,27,28,29 || exit 1
FILTER=conv_hc TAG=${T}pmc PASSES="B D X" PROBE="tools/bench_conv_vendor.py --probe 2048" \
  tools/gpu_pmc_kernels.sh > gpurun_out/${T}_pmc.txt 2>&1 || exit 1
