#!/bin/bash
# HIP-graph step capture on one MI355X: GPU tests, then eager vs graphed
# benches of a launch-bound model (LeNet / CIFAR quick) and AlexNet.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/pytest_graphs.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_graphs_gpu.py tests/test_graphs.py "tests/test_fp8.py::test_fp8_roll_kernel" || exit 1
tail -5 gpurun_out/pytest_graphs.log
for m in lenet cifar_quick; do
  tools/gpu_step.sh 300 gpurun_out/bench_${m}_eager.log env VELES_AMD_GRAPHS=0 python bench.py --model $m --batch 100 --steps 200 --warmup 10 || exit 1
  tail -1 gpurun_out/bench_${m}_eager.log
  tools/gpu_step.sh 300 gpurun_out/bench_${m}_graph.log python bench.py --model $m --batch 100 --steps 200 --warmup 10 || exit 1
  tail -1 gpurun_out/bench_${m}_graph.log
done
tools/gpu_step.sh 300 gpurun_out/bench_alexnet_eager.log env VELES_AMD_GRAPHS=0 python bench.py --steps 20 --warmup 5 || exit 1
tail -1 gpurun_out/bench_alexnet_eager.log
tools/gpu_step.sh 300 gpurun_out/bench_alexnet_graph.log python bench.py --steps 20 --warmup 5 || exit 1
tail -1 gpurun_out/bench_alexnet_graph.log
