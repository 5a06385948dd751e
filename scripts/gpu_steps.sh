#!/bin/bash
# Run GPU steps in order; each "name|timeout|command".  A failing step (rc 1: test failures) does
# not stop the rest; a timeout, abort, segfault or kill (rc 124, 134, 137, 139, >128) ends the call.
mkdir -p gpurun_out
export TMPDIR=/tmp
final=0
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; tmo=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($tmo s): $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  tail -4 "gpurun_out/$name.log"
  echo "== $name rc=$rc"
  [ $rc -ne 0 ] && final=$rc
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit $rc; fi
done
exit $final
