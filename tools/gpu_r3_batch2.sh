#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_b2.log python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "lrn or e2e or hip_matches" -m gpu -v --timeout 200 --timeout-method thread || exit 1
grep -E "passed|failed|per-layer" gpurun_out/pytest_b2.log | tail -6
tools/gpu_step.sh 200 gpurun_out/lrn_bench.log python tools/bench_lrn.py 1024 || exit 1
tail -3 gpurun_out/lrn_bench.log
tools/gpu_step.sh 300 gpurun_out/bench_b2.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_b2.log | cut -c1-150
