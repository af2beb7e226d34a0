#!/bin/bash
# ds_read_b64_tr_b8 semantics probe (built here from source), VGG-16 fp8 /
# bf16 b128 bench + fp8 step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/probes/ds_read_tr8.hip -o /tmp/ds_read_tr8 2>/dev/null || exit 1
timeout -k 10 60 /tmp/ds_read_tr8 > gpurun_out/probe_tr8.log 2>&1 || exit 1
head -20 gpurun_out/probe_tr8.log
tools/gpu_step.sh 600 gpurun_out/pytest_fp8.log python -u -m pytest tests/test_fp8.py -q -x --timeout 120 --timeout-method thread || exit 1
tail -2 gpurun_out/pytest_fp8.log
tools/gpu_step.sh 400 gpurun_out/bench_vgg_bf16.log python bench.py --model vgg16 --precision bfloat16 --steps 10 --warmup 3 --batch 128 || exit 1
grep metric gpurun_out/bench_vgg_bf16.log | cut -c1-200
BATCH=128 MODEL=vgg16 PREC=float8 TAG=r3fp8 tools/gpu_prof_step.sh
