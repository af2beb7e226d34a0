#!/bin/bash
# conv numerics + small-model benches (graphed, batch 100) + AlexNet check
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/pytest_conv.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" || exit 1
tail -3 gpurun_out/pytest_conv.log
for m in lenet cifar_quick; do
  tools/gpu_step.sh 300 gpurun_out/bench_$m.log python bench.py --model $m --batch 100 --steps 200 --warmup 10 || exit 1
  grep metric gpurun_out/bench_$m.log | cut -c1-200
done
tools/gpu_step.sh 300 gpurun_out/bench_alexnet.log python bench.py --steps 20 --warmup 5 || exit 1
grep metric gpurun_out/bench_alexnet.log | cut -c1-200
