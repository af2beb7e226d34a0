#!/bin/bash
# Whole-step A/B(/C) of environment settings on one box: bench.py alternating
# the settings A, B (and C when given), ROUNDS rounds each.
#   A="VELES_AMD_LOADER_RUNAHEAD=0" B="VELES_AMD_LOADER_RUNAHEAD=1" \
#     TAG=ra tools/gpu_bench_env_ab.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-envab}
keys="a b"; [ -n "$C" ] && keys="a b c"
for r in $(seq 1 ${ROUNDS:-3}); do
  for k in $keys; do
    case $k in a) E=$A;; b) E=$B;; c) E=$C;; esac
    env $E tools/gpu_step.sh 300 gpurun_out/${T}_${k}_$r.log \
      python3 bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-5} || exit 1
  done
done
for k in $keys; do
  case $k in a) E=$A;; b) E=$B;; c) E=$C;; esac
  echo "$k ($E): $(cat gpurun_out/${T}_${k}_*.log | grep -o '"value": [0-9.]*' | tr '\n' ' ')"
done
