#!/bin/bash
# One GPU session: smoke, 1-GPU bench, rocprofv3 kernel stats of a short run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
B=${BATCH:-512}
tools/gpu_step.sh 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tools/gpu_step.sh 600 gpurun_out/bench1.log python bench.py --steps 20 --warmup 5 --batch $B --profile-json gpurun_out/bench1_units.json || exit 1
tools/gpu_step.sh 400 gpurun_out/bk.log python tools/bench_kernels.py 512 || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh 600 gpurun_out/prof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --batch $B || exit 1
ls -R gpurun_out/prof | head -20
