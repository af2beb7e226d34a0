#!/bin/bash
# Round 6: FC weight-gradient forms at the bench batch
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6i}
tools/gpu_step.sh 300 gpurun_out/${T}_fcw.log python3 -u tools/bench_fc_wgrad_t.py 3072 5 || exit 1
