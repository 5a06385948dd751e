#!/bin/bash
U=spittle_amd/ubench; T="timeout -k 5 60"
mkdir -p gpurun_out
{
for S in 1 2 3 4; do $T $U xattn 8 1500 $S 1; done
for S in 1 2 3; do $T $U layer 8 1 $S; done
} > gpurun_out/e9.log 2>&1 || exit 1
for S in 1 2 3; do
  SPT_XATTN_SPLIT=$S timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e9_bench_$S.log 2>&1 || exit 1
  echo "xsplit=$S $(tail -1 gpurun_out/e9_bench_$S.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["roofline"]["avg_us"])')" >> gpurun_out/e9.log
done
cat gpurun_out/e9.log
