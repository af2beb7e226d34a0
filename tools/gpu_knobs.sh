#!/bin/bash
# GPU session: AlexNet bench A/B over environment knobs, interleaved twice.
# usage: KNOBS="A=1 B=0;C=1" bash tools/gpu_knobs.sh   (";" separates settings,
# the empty setting = defaults is always run first)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
IFS=';' read -ra SETS <<< ";${KNOBS}"
for rep in 1 2; do
  i=0
  for kv in "${SETS[@]}"; do
    env $kv tools/gpu_step.sh 300 gpurun_out/knob_${i}_$rep.log python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} || exit 1
    echo "[$kv] $(grep -h -o '"value": [0-9.]*' gpurun_out/knob_${i}_$rep.log)"
    i=$((i+1))
  done
done
