#!/bin/bash
# GPU session: the multi-rank bench path rehearsed with 2 ranks on the one
# GPU of a gpurun box (gloo carries the gradient all-reduce: RCCL refuses two
# ranks on one device), the RCCL all-reduce microbench at world 1, and the
# VGG-16 bf16 / fp8 benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
VELES_AMD_DP_BACKEND=gloo tools/gpu_step.sh 400 gpurun_out/dp2_gloo.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --batch 256 || exit 1
tail -2 gpurun_out/dp2_gloo.log
tools/gpu_step.sh 200 gpurun_out/allreduce1.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 tools/bench_allreduce.py || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_bf16.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
tools/gpu_step.sh 400 gpurun_out/vgg_fp8.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision float8 || exit 1
