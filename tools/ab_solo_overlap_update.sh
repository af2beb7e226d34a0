#!/bin/bash
# The multi-rank step through a one-rank RCCL group, backward eager (the
# N > 1 default): per-bucket updates overlapped on the side stream (1, the
# default) or one update after the last all-reduce (0), alternating
set -e
export VELES_AMD_DP_SOLO_COLLECTIVES=1 VELES_AMD_DP_GRAPH_BACKWARD=0
p=29570
for i in 1 2; do
  for v in 1 0; do
    p=$((p+1))
    VELES_AMD_DP_OVERLAP_UPDATE=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/solo_ou${v}_$i.log 2>&1
    echo "overlap_update=$v run $i: $(grep -ho '"value": [0-9.]*' gpurun_out/solo_ou${v}_$i.log)"
  done
done
