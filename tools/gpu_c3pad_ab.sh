#!/bin/bash
# GPU session: conv numerics with the channel-padding path, then VGG-16 b128
# (bf16) and CIFAR quick b4096 with HVK_C3_PAD=1 (default) and =0, twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/conv_tests.log python -u -m pytest tests/test_kernels_gpu.py tests/test_graphs_gpu.py -k "conv or graph" -x -q --timeout 120 --timeout-method thread || exit 1
tail -2 gpurun_out/conv_tests.log
for r in 1 2; do for p in 1 0; do
HVK_C3_PAD=$p tools/gpu_step.sh 300 gpurun_out/vgg_pad${p}_$r.log python bench.py --model vgg16 --batch 128 --steps 10 --warmup 3 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/vgg_pad${p}_$r.log | sed "s/^/vgg16 bf16 pad=$p: /"
HVK_C3_PAD=$p tools/gpu_step.sh 300 gpurun_out/cifar_pad${p}_$r.log python bench.py --model cifar_quick --batch 4096 --steps 20 --warmup 5 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/cifar_pad${p}_$r.log | sed "s/^/cifar pad=$p: /"
done; done
