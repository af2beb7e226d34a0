#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
tools/gpu_r3_batch3.sh || exit 1
tools/gpu_r3_mf32.sh
