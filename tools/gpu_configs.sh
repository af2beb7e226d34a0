#!/bin/bash
# GPU session: every BASELINE.json configuration on one MI355X.
#  1 MNIST all2all on the CPU device (numpy-backend analogue)
#  2 LeNet-style MNIST convnet, bf16       3 CIFAR-10 quick convnet, bf16
#  4 AlexNet (bench.py default)            5 VGG-16 fp8
# plus two sample workflows end to end through the CLI (train + snapshot).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/cfg
tools/gpu_step.sh 300 gpurun_out/cfg/c1_mnist_fc_cpu.log python bench.py --cpu --model mnist_fc --batch 100 --steps 20 --warmup 3 || exit 1
tools/gpu_step.sh 300 gpurun_out/cfg/c2_lenet.log python bench.py --model lenet --batch 4096 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 gpurun_out/cfg/c3_cifar_quick.log python bench.py --model cifar_quick --batch 4096 --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 300 gpurun_out/cfg/c4_alexnet.log python bench.py --steps 20 --warmup 5 || exit 1
tools/gpu_step.sh 400 gpurun_out/cfg/c5_vgg16_fp8.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 --precision float8 || exit 1
tools/gpu_step.sh 300 gpurun_out/cfg/wf_mnist_conv.log python -m veles_amd samples/mnist_conv.py - 'root.common.dirs.snapshots="gpurun_out/cfg/snap"' || exit 1
tools/gpu_step.sh 300 gpurun_out/cfg/wf_cifar_conv.log python -m veles_amd samples/cifar_conv.py - 'root.common.dirs.snapshots="gpurun_out/cfg/snap"' || exit 1
for f in gpurun_out/cfg/*.log; do echo "== $f"; tail -n 2 "$f"; done
