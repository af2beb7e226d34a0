#!/bin/bash
# split-K partial sums in per-split workspace slices: numerics, FC A/B, bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_splitk.log python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_pp_gpu.py tests/test_e2e_gpu.py -q -x --timeout 120 --timeout-method thread -k "gemm or splitk or fc or all2all or e2e or pp" || exit 1
tail -2 gpurun_out/pytest_splitk.log
grep -q " passed" gpurun_out/pytest_splitk.log && ! grep -q "FAILED\| failed" gpurun_out/pytest_splitk.log || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_splitk.log | head -60; exit 1; }
tools/gpu_step.sh 300 gpurun_out/fc_ab_slices.log python tools/bench_fc_ab.py 1024 5 || exit 1
grep -v "^\[" gpurun_out/fc_ab_slices.log | grep ours
tools/gpu_step.sh 300 gpurun_out/bench_splitk.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_splitk.log | cut -c1-170
