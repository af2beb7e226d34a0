#!/bin/bash
# Whole-step A/B of two kernel libraries on one box: bench.py alternating
# the shipped libhvk.so and $EXP (HVK_LIBRARY), ROUNDS rounds each.
#   EXP=build/ab/libhvk_x.so TAG=ab tools/gpu_bench_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-benchab}
for r in $(seq 1 ${ROUNDS:-3}); do
  tools/gpu_step.sh 300 gpurun_out/${T}_new_$r.log python3 bench.py --steps 30 --warmup 5 || exit 1
  HVK_LIBRARY=$EXP tools/gpu_step.sh 300 gpurun_out/${T}_exp_$r.log python3 bench.py --steps 30 --warmup 5 || exit 1
done
for k in new exp; do
  echo "$k: $(cat gpurun_out/${T}_${k}_*.log | grep -o '"value": [0-9.]*' | tr '\n' ' ')"
done
