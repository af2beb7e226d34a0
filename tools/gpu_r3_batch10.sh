#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/pytest_b10.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "gemm or conv or lrn" || exit 1
tail -2 gpurun_out/pytest_b10.log
grep -q " passed" gpurun_out/pytest_b10.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_b10.log || exit 1
tools/gpu_step.sh 300 gpurun_out/lrn_ab3.log python tools/bench_lrn.py 1024 || exit 1
grep "bwd" gpurun_out/lrn_ab3.log | grep -v "^{" | tail -3
# grouped tile order (-1) vs row-major (20)
tools/gpu_step.sh 400 gpurun_out/ab_grouped.log python tools/bench_gemm_ab.py 1024 5 -1,20 || exit 1
grep -v "^\[" gpurun_out/ab_grouped.log | head -24
tools/gpu_step.sh 300 gpurun_out/bench_b10.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_b10.log | cut -c1-200
