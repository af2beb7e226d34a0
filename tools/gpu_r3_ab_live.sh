#!/bin/bash
# A/B of the GEMM dead-wave skip: shipped library (no skip) vs build/ab/libhvk_live.so, A B A
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/ab_nolive1.log python tools/bench_gemm_ab.py 1024 3 -1 || exit 1
HVK_LIBRARY=$R/build/ab/libhvk_live.so tools/gpu_step.sh 300 gpurun_out/ab_live.log python tools/bench_gemm_ab.py 1024 3 -1 || exit 1
tools/gpu_step.sh 300 gpurun_out/ab_nolive2.log python tools/bench_gemm_ab.py 1024 3 -1 || exit 1
paste <(grep -v "^\[" gpurun_out/ab_nolive1.log | grep TF) <(grep -v "^\[" gpurun_out/ab_live.log | grep TF | awk '{print $2}') <(grep -v "^\[" gpurun_out/ab_nolive2.log | grep TF | awk '{print $2}')
tools/gpu_step.sh 300 gpurun_out/bench_nolive.log python bench.py --steps 20 --warmup 5 || exit 1
HVK_LIBRARY=$R/build/ab/libhvk_live.so tools/gpu_step.sh 300 gpurun_out/bench_live.log python bench.py --steps 20 --warmup 5 || exit 1
grep -h metric gpurun_out/bench_nolive.log gpurun_out/bench_live.log | cut -c1-170
