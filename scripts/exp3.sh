#!/bin/bash
# parity tests, then decoder microbenchmarks of the 6-launch layer, then the bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e3_tests.log 2>&1; rc=$?
tail -5 gpurun_out/e3_tests.log
[ $rc -le 1 ] || exit $rc
U=spittle_amd/ubench; T="timeout -k 5 60"
{
$T $U layer 8 1 2 - 2 2 4
$T $U layer 8 1 1 - 1 1 1
$T $U layer 8 1 3 - 2 2 4
$T $U layer 8 1 2 - 1 1 4
$T $U layer 8 1 2 - 2 2 2
for S in 1 2 3 4; do $T $U xattn 8 1500 $S 1 1; done
$T $U gemv 1280 1280 8 2 0 1 1
$T $U gemv 1280 1280 8 2 0 1 2
$T $U gemv 1280 5120 8 2 0 1 1
$T $U gemv 1280 5120 8 2 0 1 4
$T $U gemv 5120 1280 8 1 1 1
$T $U gemv 3840 1280 8 3 1 1
$T $U attn 8 20 448 132 1 1
} > gpurun_out/e3_ubench.log 2>&1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e3_bench.log 2>&1; tail -1 gpurun_out/e3_bench.log
