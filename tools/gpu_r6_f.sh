#!/bin/bash
# Round 6: exact-resume tests (deterministic mode), AlexNet b3072 step
# profiles (overlapped and serialised), VGG-16 b512 bf16 / fp8 benches
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6f}
tools/gpu_step.sh 400 gpurun_out/${T}_resume.log python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_resume_gpu.py -s || exit 1
tools/gpu_step.sh 400 gpurun_out/${T}_prof.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
AMD_SERIALIZE_KERNEL=3 tools/gpu_step.sh 400 gpurun_out/${T}_prof_serial.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_serial" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --mark-steps || exit 1
for f in $(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1); do python3 tools/prof_summary.py "$f" gpurun_out/${T}_step.md "alexnet b3072 1x MI355X (bf16, ${T})" --window --steps 5; done
for f in $(find gpurun_out/${T}_prof_serial -name "*kernel_trace.csv" | head -1); do python3 tools/prof_summary.py "$f" gpurun_out/${T}_step_serial.md "alexnet b3072 1x MI355X (bf16, ${T}, serialised)" --window --steps 5; done
tools/gpu_step.sh 400 gpurun_out/${T}_vgg_bf16.log python3 bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
tools/gpu_step.sh 400 gpurun_out/${T}_vgg_fp8.log python3 bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
