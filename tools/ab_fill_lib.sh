#!/bin/bash
# tools/probe_fill_s2d.py with another revision's elementwise.hip
# (abl/libhvk_fill_old.so: python tools/build_ab_lib.py elementwise HEAD
# abl/libhvk_fill_old.so) against the working tree's, alternating on one box
set -e
for i in 1 2 3; do
  HVK_LIBRARY=abl/libhvk_fill_old.so timeout -k 10 120 python tools/probe_fill_s2d.py 2048 > gpurun_out/fill_old_$i.log 2>&1
  timeout -k 10 120 python tools/probe_fill_s2d.py 2048 > gpurun_out/fill_new_$i.log 2>&1
  for v in old new; do echo "$v $i: $(grep -h '^fill' gpurun_out/fill_${v}_$i.log)"; done
done
