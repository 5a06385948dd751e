#!/bin/bash
# gpurun that waits for a free box: retries ONLY while gpurun answers 3 (no box / slot free, nothing
# ran); any other outcome (including a failing command) is final.  usage: gpurun_wait.sh OUT TIMEOUT CMD
out=$1; tmo=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "gpurun_rc=$rc" >> "$out"
