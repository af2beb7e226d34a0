#!/bin/bash
# Round-5 fp8 halo wgrad: fp8 + halo tests, the fp8 kernel A/B on VGG shapes,
# then the VGG-16 b512 fp8 step on / off.  usage: TAG=r5c tools/gpu_r5_fp8.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
S=tools/gpu_step.sh
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8.py tests/test_wgrad_halo_gpu.py -m gpu > gpurun_out/fp8_test_${T}.log 2>&1 || { tail -40 gpurun_out/fp8_test_${T}.log; exit 1; }
tail -3 gpurun_out/fp8_test_${T}.log
timeout -k 10 600 python -u tools/bench_wgrad8_ab.py 512 5 > gpurun_out/halo8_ab_${T}.log 2>&1 || { tail gpurun_out/halo8_ab_${T}.log; exit 1; }
cat gpurun_out/halo8_ab_${T}.log
if [ -n "$STEP" ]; then
$S 600 gpurun_out/bench_vgg8_${T}_on.log python bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
VELES_AMD_HALO_WGRAD=0 $S 600 gpurun_out/bench_vgg8_${T}_off.log python bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
$S 600 gpurun_out/bench_vgg16_${T}_on.log python bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
grep -h '^{' gpurun_out/bench_vgg8_${T}_*.log gpurun_out/bench_vgg16_${T}_on.log | cut -c1-200
export TMPDIR=/tmp
$S 600 gpurun_out/prof_vgg8_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vgg8_${T}" -o run --output-format csv -- python3 "$R/bench.py" --model vgg16 --precision float8 --steps 3 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_vgg8_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_vgg8_${T}.md "vgg16 b512 1x MI355X (float8, $T)" --window --steps 3
rm -rf gpurun_out/prof_vgg8_${T}
fi
exit 0
