#!/bin/bash
# VGG-16 b128 bf16 vs fp8 benches + fp8 kernel profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for p in bfloat16 float8; do
  tools/gpu_step.sh 400 gpurun_out/bench_vgg_$p.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision $p || exit 1
  grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/bench_vgg_$p.log
done
tools/gpu_step.sh 600 gpurun_out/prof_vgg8.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg8" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --batch 128 --model vgg16 --precision float8 || exit 1
