#!/bin/bash
# LeNet / CIFAR quick b100: weight gradients on branch streams (default) vs
# serial (VELES_AMD_WGRAD_STREAM=0), alternating on one box
set -e
mkdir -p gpurun_out/ab_small
for i in 1 2; do
  for m in lenet cifar_quick; do
    for ws in default 0; do
      if [ $ws = 0 ]; then export VELES_AMD_WGRAD_STREAM=0; else unset VELES_AMD_WGRAD_STREAM; fi
      timeout -k 10 120 python -u bench.py --model $m --batch 100 --steps 200 --warmup 20 > gpurun_out/ab_small/${m}_${ws}_$i.log 2>&1
      echo "$m wgrad_stream=$ws run $i: $(grep -ho '"value": [0-9.]*' gpurun_out/ab_small/${m}_${ws}_$i.log)"
    done
  done
done
