#!/bin/bash
# Round-5 checkpoint: GPU tests touched this round, AlexNet bench x2 and
# step profile with the current defaults.  usage: TAG=r5i tools/gpu_r5_base.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r5}
S=tools/gpu_step.sh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgrad_halo_gpu.py tests/test_conv_ws_gpu.py tests/test_branch_streams_gpu.py tests/test_graphs_gpu.py tests/test_e2e_gpu.py -m gpu > gpurun_out/tests_${T}.log 2>&1 || { tail -40 gpurun_out/tests_${T}.log; exit 1; }
tail -3 gpurun_out/tests_${T}.log
$S 400 gpurun_out/bench_alex_${T}_1.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 gpurun_out/bench_alex_${T}_2.log python bench.py --steps 20 --warmup 5 || exit 1
grep -h '^{' gpurun_out/bench_alex_${T}_*.log | cut -c1-200
export TMPDIR=/tmp
$S 600 gpurun_out/prof_alex_${T}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_alex_${T}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
f=$(find gpurun_out/prof_alex_${T} -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py "$f" gpurun_out/prof_alex_${T}.md "alexnet b2048 1x MI355X (bfloat16, $T)" --window --steps 5
rm -rf gpurun_out/prof_alex_${T}
head -30 gpurun_out/prof_alex_${T}.md
