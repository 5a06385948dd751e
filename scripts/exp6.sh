#!/bin/bash
mkdir -p gpurun_out
for pf in 0 1 2; do
  for wg in 64 256; do
    [ $pf -eq 0 ] && [ $wg -eq 256 ] && continue
    SPT_PREFETCH=$pf SPT_PREFETCH_WG=$wg timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e6_bench_$pf_$wg.log 2>&1 || exit 1
    echo "prefetch=$pf wg=$wg $(tail -1 gpurun_out/e6_bench_$pf_$wg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"])')"
  done
done
