#!/bin/bash
# Host-ASan build of the native runtime self-tests, run on the GPU box
# (GPU code unsanitized: -fno-gpu-sanitize), including the branch-stream /
# hipGraph test.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
python -c "
from veles_amd.runtime import build_sanitized_tests
exe, env = build_sanitized_tests('asan')
print(exe)
" > gpurun_out/asan_build.log 2>&1 || { cat gpurun_out/asan_build.log; exit 1; }
EXE=$(tail -1 gpurun_out/asan_build.log)
export ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0:abort_on_error=0
timeout -k 10 120 "$EXE" --gpu-branch > gpurun_out/asan_gpu_branch.log 2>&1
echo "rc=$?" >> gpurun_out/asan_gpu_branch.log
tail -40 gpurun_out/asan_gpu_branch.log
