#!/bin/bash
# 2-rank data-parallel rehearsal on one GPU (gloo: RCCL refuses two ranks on
# one device) + the 1-rank RCCL launch path the driver uses
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
VELES_AMD_DP_BACKEND=gloo tools/gpu_step.sh 400 gpurun_out/dp2_gloo.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 3 --batch 256 || exit 1
grep -h metric gpurun_out/dp2_gloo.log | cut -c1-400
tools/gpu_step.sh 300 gpurun_out/dp1_nccl.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
grep -h metric gpurun_out/dp1_nccl.log | cut -c1-600
