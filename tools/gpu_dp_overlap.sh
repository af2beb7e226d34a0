#!/bin/bash
# GPU session: the per-bucket overlapped update (ParameterStore._bucket_update)
# on a real GPU - the two-rank numerics test (gloo collectives, overlap
# forced), then the multi-rank gradient path under RCCL stream semantics on
# one GPU: a one-rank RCCL process group (VELES_AMD_DP_SOLO_COLLECTIVES=1)
# with the overlap on and off, against the plain single-GPU step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/dp_overlap_test.log python -u -m pytest tests/test_dp_gloo.py -m gpu -x -v --timeout 250 --timeout-method thread || exit 1
tail -3 gpurun_out/dp_overlap_test.log
for r in 1 2; do
for ov in 1 0; do
VELES_AMD_DP_OVERLAP_UPDATE=$ov VELES_AMD_DP_SOLO_COLLECTIVES=1 MASTER_PORT=2955$ov tools/gpu_step.sh 300 gpurun_out/solo_ov${ov}_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/solo_ov${ov}_$r.log | sed "s/^/solo overlap=$ov: /"
done
tools/gpu_step.sh 300 gpurun_out/plain_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/plain_$r.log | sed "s/^/plain: /"
done
