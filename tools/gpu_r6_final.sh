#!/bin/bash
# Round 6 final: GPU suite, smoke, bench x2, serialised step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6fin}
bash tools/gpu_full.sh || exit 1
tools/gpu_step.sh 300 gpurun_out/${T}_bench2.log python3 bench.py --steps 40 --warmup 5 || exit 1
AMD_SERIALIZE_KERNEL=3 tools/gpu_step.sh 400 gpurun_out/${T}_prof_serial.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_serial" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
for f in $(find gpurun_out/${T}_prof_serial -name "*kernel_trace.csv" | head -1); do python3 tools/prof_summary.py "$f" gpurun_out/${T}_step_serial.md "alexnet b3072 1x MI355X (bf16, ${T}, serialised)" --window --steps 5; done
tools/gpu_step.sh 400 gpurun_out/${T}_vgg_bf16.log python3 bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
tools/gpu_step.sh 400 gpurun_out/${T}_vgg_fp8.log python3 bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
