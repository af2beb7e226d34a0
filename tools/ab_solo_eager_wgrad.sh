#!/bin/bash
# The multi-rank step through a one-rank RCCL group, backward eager (the
# N > 1 default): weight gradients on branch streams (1) or serial (0)
set -e
export VELES_AMD_DP_SOLO_COLLECTIVES=1 VELES_AMD_DP_GRAPH_BACKWARD=0
p=29550
for i in 1 2; do
  for v in 1 0; do
    p=$((p+1))
    VELES_AMD_WGRAD_STREAM=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/solo_eager_ws${v}_$i.log 2>&1
    echo "wgrad_stream=$v run $i: $(grep -ho '"value": [0-9.]*' gpurun_out/solo_eager_ws${v}_$i.log)"
  done
done
