#!/bin/bash
# rocprofv3 kernel stats of short VGG-16 runs (bf16 and fp8).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/prof_vgg8.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg8" -o run --output-format csv -- python3 "$R/bench.py" --model vgg16 --batch 128 --steps 3 --warmup 2 --precision float8 || exit 1
tools/gpu_step.sh 400 gpurun_out/prof_vgg16.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg16" -o run --output-format csv -- python3 "$R/bench.py" --model vgg16 --batch 128 --steps 3 --warmup 2 || exit 1
