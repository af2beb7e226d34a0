#!/bin/bash
# A/B of the side-stream bucket update grid (VELES_AMD_DP_UPDATE_BLOCKS) under
# a one-rank RCCL process group (the multi-rank gradient path on one GPU),
# against the fused update after the backward and the plain single-GPU step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
if [ -n "$CFG_LIST" ]; then IFS=',' read -ra CFGS <<< "$CFG_LIST"
else CFGS=("1 0" "1 32" "1 64" "1 128" "1 256" "0 0"); fi
for r in 1 2; do
for cfg in "${CFGS[@]}"; do
set -- $cfg
VELES_AMD_DP_OVERLAP_UPDATE=$1 VELES_AMD_DP_UPDATE_BLOCKS=$2 VELES_AMD_DP_SOLO_COLLECTIVES=1 MASTER_PORT=2956$r tools/gpu_step.sh 300 gpurun_out/solo_ov$1_b$2_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/solo_ov$1_b$2_$r.log | sed "s/^/solo overlap=$1 blocks=$2: /"
done
tools/gpu_step.sh 300 gpurun_out/plain_$r.log python bench.py --steps 20 --warmup 5 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/plain_$r.log | sed "s/^/plain: /"
done
