#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/cfg/snap
grep "wf_" tools/gpu_configs.sh | grep -v "^for" > /tmp/wf_steps.sh
bash -e /tmp/wf_steps.sh
for f in gpurun_out/cfg/wf_*.log; do echo "== $f"; tail -n 6 "$f"; done
ls gpurun_out/cfg/snap | head
