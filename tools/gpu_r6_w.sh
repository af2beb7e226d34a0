#!/bin/bash
# Round 6: VGG-16 b512 serialised step profiles, fp8 and bf16
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6w}
for P in float8 bfloat16; do
AMD_SERIALIZE_KERNEL=3 tools/gpu_step.sh 400 gpurun_out/${T}_${P}.log rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_${P}" -o run --output-format csv -- python3 "$R/bench.py" --model vgg16 --precision $P --steps 3 --warmup 2 --mark-steps || exit 1
for f in $(find gpurun_out/${T}_${P} -name "*kernel_trace.csv" | head -1); do python3 tools/prof_summary.py "$f" gpurun_out/${T}_vgg_${P}.md "vgg16 b512 1x MI355X (${P}, ${T}, serialised)" --window --steps 3; done
done
