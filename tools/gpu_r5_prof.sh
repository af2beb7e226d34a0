#!/bin/bash
# Step-only rocprofv3 kernel summary of the AlexNet b2048 bench (and, with
# VGG=1, VGG-16 b512 bf16 / fp8 bench lines).  usage: TAG=r5l tools/gpu_r5_prof.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
S=tools/gpu_step.sh
export TMPDIR=/tmp
$S 600 gpurun_out/prof_alex_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_alex_${T}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_alex_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_alex_${T}.md "alexnet b2048 1x MI355X (bfloat16, $T)" --window --steps 5
rm -rf gpurun_out/prof_alex_${T}
if [ -n "$VGG" ]; then
$S 600 gpurun_out/bench_vgg_${T}_bf16.log python bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
$S 600 gpurun_out/bench_vgg_${T}_fp8.log python bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
grep -h '^{' gpurun_out/bench_vgg_${T}_*.log | cut -c1-200
fi
