#!/bin/bash
# the other BASELINE configs on the round-3 build: LeNet / CIFAR quick at
# b4096 and b100, VGG-16 bf16 / fp8 b128, mnist_fc
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/configs_r3
export TMPDIR=/tmp
for cfg in "lenet 4096" "lenet 100" "cifar_quick 4096" "cifar_quick 100" "mnist_fc 4096"; do
  set -- $cfg
  tools/gpu_step.sh 300 gpurun_out/configs_r3/$1_b$2.log python bench.py --model $1 --batch $2 --steps 50 --warmup 10 || exit 1
  grep -h metric gpurun_out/configs_r3/$1_b$2.log | cut -c1-160
done
for p in bfloat16 float8; do
  tools/gpu_step.sh 400 gpurun_out/configs_r3/vgg16_$p.log python bench.py --model vgg16 --precision $p --batch 128 --steps 20 --warmup 5 || exit 1
  grep -h metric gpurun_out/configs_r3/vgg16_$p.log | cut -c1-160
done
