#!/bin/bash
# conv_ws ablation: kernel A/B with HVK_WS_ABL = 0 / 1 / 2 / 4 / 7
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for a in 0 1 2 4 3; do
  echo "== HVK_WS_ABL=$a"
  HVK_WS_ABL=$a timeout -k 10 300 python -u tools/bench_conv_ab.py 2048 3 128 > gpurun_out/ws_abl_$a.log 2>&1 || { tail gpurun_out/ws_abl_$a.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ws_abl_$a.log
done
for a in 0 1 2 4; do
  echo "== HVK_HALO_ABL=$a"
  HVK_HALO_ABL=$a timeout -k 10 300 python -u tools/bench_wgrad_ab.py 2048 3 > gpurun_out/halo_abl_$a.log 2>&1 || { tail gpurun_out/halo_abl_$a.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/halo_abl_$a.log
done
