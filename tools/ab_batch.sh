#!/bin/bash
# AlexNet bench at per-GPU batch 2048 / 3072 / 4096, alternating on one box
set -e
for i in 1 2; do
  for b in ${BATCHES:-2048 3072 4096}; do
    timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/b_batch${b}_$i.log 2>&1
    echo "batch=$b run $i: $(grep -ho '"value": [0-9.]*' gpurun_out/b_batch${b}_$i.log)"
  done
done
