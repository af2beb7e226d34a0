#!/bin/bash
# LRN->pool forward walk kernel: numerics, A/B timing, AlexNet bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_lrn.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "lrn" || exit 1
tail -3 gpurun_out/pytest_lrn.log
tools/gpu_step.sh 300 gpurun_out/lrn_ab.log python tools/bench_lrn.py 1024 || exit 1
grep -v "^\[" gpurun_out/lrn_ab.log | tail -6
tools/gpu_step.sh 300 gpurun_out/bench_lrnwalk.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_lrnwalk.log | cut -c1-200
