#!/bin/bash
# GPU session: tuning-table test, the autotuner over AlexNet b512 (table
# written to gpurun_out/gfx950.json, copied to devices/ afterwards), then the
# AlexNet bench with the tuned table and without (VELES_AMD_TUNING=0), twice.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 200 gpurun_out/autotune_test.log python -u -m pytest tests/test_autotune.py -m gpu -x -v --timeout 150 --timeout-method thread || exit 1
tail -2 gpurun_out/autotune_test.log
tools/gpu_step.sh 400 gpurun_out/autotune.log python -u -m veles_amd.ops.autotune --model ${MODELS:-alexnet} --batch ${BATCH:-512} --out gpurun_out/gfx950.json || exit 1
cat gpurun_out/autotune.log
for r in 1 2; do
VELES_AMD_TUNING_FILE=gpurun_out/gfx950.json tools/gpu_step.sh 300 gpurun_out/bench_tuned_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tuned_$r.log | sed "s/^/tuned: /"
VELES_AMD_TUNING=0 tools/gpu_step.sh 300 gpurun_out/bench_untuned_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_untuned_$r.log | sed "s/^/untuned: /"
done
