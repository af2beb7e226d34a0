#!/bin/bash
# multi-rank bench path (2 ranks via gloo on the one GPU) and a one-rank RCCL
# group through torch.distributed.run - the driver's N > 1 launch path
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
VELES_AMD_DP_BACKEND=gloo tools/gpu_step.sh 400 gpurun_out/dp2_gloo_r3.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --batch 256 || exit 1
grep metric gpurun_out/dp2_gloo_r3.log | cut -c1-400
tools/gpu_step.sh 400 gpurun_out/dp1_rccl_r3.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/dp1_rccl_r3.log | cut -c1-600
