#!/bin/bash
# Round 6: conv_hc32 with packed weights - numerics, bench-scale gate,
# ablation, A/B, PMC (cache / traffic), bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6c}
tools/gpu_step.sh 600 gpurun_out/${T}_pytest.log python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_conv_hc_gpu.py tests/test_alexnet_bench_scale_gpu.py tests/test_graphs_gpu.py -s || exit 1
tools/gpu_step.sh 300 gpurun_out/${T}_bench.log python3 bench.py || exit 1
tools/gpu_step.sh 400 gpurun_out/${T}_ab.log python3 -u tools/bench_conv_hc_ab.py 2048 3 || exit 1
if [ -f build/hcabl/libhvk_hcabl.so ]; then
  HVK_LIBRARY=build/hcabl/libhvk_hcabl.so tools/gpu_step.sh 400 gpurun_out/${T}_abl.log python3 -u tools/ablate_conv_hc.py 2048 3 || exit 1
fi
FILTER=conv_hc TAG=${T}pmc PASSES="B M L F" PROBE="tools/bench_conv_vendor.py --probe 2048" \
  tools/gpu_pmc_kernels.sh > gpurun_out/${T}_pmc.txt 2>&1 || exit 1
