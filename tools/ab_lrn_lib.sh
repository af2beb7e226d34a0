#!/bin/bash
# bench_lrn.py with an older pool_lrn.hip (abl/libhvk_lrn_old.so, e.g.
#   python tools/build_ab_lib.py pool_lrn 55a0089 abl/libhvk_lrn_old.so \
#       --stub hvk_set_pool_bwd_variant)
# against the working tree's, alternating on one box
set -e
for i in 1 2; do
  HVK_LIBRARY=abl/libhvk_lrn_old.so timeout -k 10 200 python tools/bench_lrn.py 2048 > gpurun_out/lrn_old_$i.log 2>&1
  timeout -k 10 200 python tools/bench_lrn.py 2048 > gpurun_out/lrn_new_$i.log 2>&1
  for v in old new; do echo "$v $i: $(grep -h "^conv. {" gpurun_out/lrn_${v}_$i.log | tr '\n' ' ')"; done
done
