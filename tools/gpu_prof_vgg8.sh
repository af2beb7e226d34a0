#!/bin/bash
# GPU session: rocprofv3 kernel stats of VGG-16 b128 fp8 and bf16 bench runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/prof_vgg8.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg8" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --batch 128 --model vgg16 --precision float8 || exit 1
tools/gpu_step.sh 600 gpurun_out/prof_vgg16.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg16" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --batch 128 --model vgg16 || exit 1
