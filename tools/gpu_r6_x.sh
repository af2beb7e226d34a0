#!/bin/bash
# Round 6: VGG-16 b512 fp8 with conv1_2 on bf16 (default) vs every eligible
# conv on fp8 (VELES_AMD_FP8_ALL_CONVS=1), alternating on one box; bf16 ref
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r6x}
for r in 1 2; do
  tools/gpu_step.sh 400 gpurun_out/${T}_fp8_$r.log python3 bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
  VELES_AMD_FP8_ALL_CONVS=1 tools/gpu_step.sh 400 gpurun_out/${T}_fp8all_$r.log python3 bench.py --model vgg16 --precision float8 --steps 10 --warmup 4 || exit 1
done
tools/gpu_step.sh 400 gpurun_out/${T}_bf16.log python3 bench.py --model vgg16 --steps 10 --warmup 4 || exit 1
for k in fp8 fp8all bf16; do
  echo "$k: $(cat gpurun_out/${T}_${k}_*.log gpurun_out/${T}_${k}.log 2>/dev/null | grep -o '"value": [0-9.]*' | tr '\n' ' ')"
done
