#!/bin/bash
# AlexNet b2048: conv weight gradients forked before (0) or after (1) the
# layer's backward-data, alternating on one box
set -e
for i in 1 2; do
  for v in 0 1; do
    VELES_AMD_WGRAD_AFTER=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_after${v}_$i.log 2>&1
    echo "after=$v run $i: $(grep -ho '"value": [0-9.]*' gpurun_out/b_after${v}_$i.log)"
  done
done
