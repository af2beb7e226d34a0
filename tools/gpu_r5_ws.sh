#!/bin/bash
# Round-5 weight-stationary convs: numerics tests, kernel A/B, AlexNet step
# A/B + profile.  usage: TAG=r5d STEP=1 tools/gpu_r5_ws.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
S=tools/gpu_step.sh
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_ws_gpu.py > gpurun_out/ws_test_${T}.log 2>&1 || { tail -40 gpurun_out/ws_test_${T}.log; exit 1; }
tail -3 gpurun_out/ws_test_${T}.log
timeout -k 10 600 python -u tools/bench_conv_ab.py 2048 5 128 > gpurun_out/ws_ab_${T}.log 2>&1 || { tail gpurun_out/ws_ab_${T}.log; exit 1; }
cat gpurun_out/ws_ab_${T}.log
if [ -n "$STEP" ]; then
$S 400 gpurun_out/bench_alex_${T}_on1.log python bench.py --steps 20 --warmup 5 || exit 1
VELES_AMD_CONV_WS=0 $S 400 gpurun_out/bench_alex_${T}_off.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 gpurun_out/bench_alex_${T}_on2.log python bench.py --steps 20 --warmup 5 || exit 1
grep -h '^{' gpurun_out/bench_alex_${T}_*.log | cut -c1-200
export TMPDIR=/tmp
$S 600 gpurun_out/prof_alex_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_alex_${T}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_alex_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_alex_${T}.md "alexnet b2048 1x MI355X (bfloat16, $T)" --window --steps 5
rm -rf gpurun_out/prof_alex_${T}
fi
exit 0
