#!/bin/bash
# Round-5 step A/B: AlexNet b2048 with the halo weight gradient on / off /
# on (same box), step-only rocprofv3 summary with it on, VGG-16 b512 bf16
# on / off.  usage: TAG=r5a tools/gpu_r5_step.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
S=tools/gpu_step.sh
$S 400 gpurun_out/bench_alex_${T}_on1.log python bench.py --steps 20 --warmup 5 || exit 1
VELES_AMD_HALO_WGRAD=0 $S 400 gpurun_out/bench_alex_${T}_off.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 gpurun_out/bench_alex_${T}_on2.log python bench.py --steps 20 --warmup 5 || exit 1
grep -h '^{' gpurun_out/bench_alex_${T}_*.log | cut -c1-200
export TMPDIR=/tmp
$S 600 gpurun_out/prof_alex_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_alex_${T}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_alex_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_alex_${T}.md "alexnet b2048 1x MI355X (bfloat16, $T)" --window --steps 5
rm -rf gpurun_out/prof_alex_${T}
if [ -n "$VGG" ]; then
$S 600 gpurun_out/bench_vgg_${T}_on.log python bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
VELES_AMD_HALO_WGRAD=0 $S 600 gpurun_out/bench_vgg_${T}_off.log python bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
grep -h '^{' gpurun_out/bench_vgg_${T}_*.log | cut -c1-200
fi
