#!/bin/bash
# rocprofv3 memory-side PMC passes on a short AlexNet bench (one counter
# group per run, kernel-trace only): HBM fetch bytes + TA busy, then HBM
# write bytes + L2 hit / miss.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc2" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmc2.log 2>&1 || exit 1
echo "pmc2 ok"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/pmc3" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > gpurun_out/pmc3.log 2>&1 || exit 1
echo "pmc3 ok"
