#!/bin/bash
# The smaller BASELINE configs (MNIST FC, LeNet, CIFAR quick) and VGG-16 on
# one MI355X, each bench under its own time limit; logs to gpurun_out/configs_r5/
set -e
mkdir -p gpurun_out/configs_r5
run() {
  local name=$1; shift
  timeout -k 10 240 python -u bench.py "$@" > gpurun_out/configs_r5/$name.log 2>&1
  echo "$name: $(grep -ho '"value": [0-9.]*' gpurun_out/configs_r5/$name.log)"
}
run mnist_fc_b4096 --model mnist_fc --batch 4096 --steps 50 --warmup 10
run lenet_b4096 --model lenet --batch 4096 --steps 50 --warmup 10
run lenet_b100 --model lenet --batch 100 --steps 50 --warmup 10
run cifar_quick_b4096 --model cifar_quick --batch 4096 --steps 50 --warmup 10
run cifar_quick_b100 --model cifar_quick --batch 100 --steps 50 --warmup 10
run vgg16_bf16_b512 --model vgg16 --steps 10 --warmup 3
run vgg16_fp8_b512 --model vgg16 --precision float8 --steps 10 --warmup 3
