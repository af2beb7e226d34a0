#!/bin/bash
# Run one GPU step under a time limit; stop the whole call on a fault,
# abort, segfault or timeout (exit codes >= 124), tolerate plain test
# failures (rc 1) so that later steps still run.
# usage: tools/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$log"
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
  echo "[gpu_step] FATAL rc=$rc in: $*" >&2
  exit 99
fi
exit 0
