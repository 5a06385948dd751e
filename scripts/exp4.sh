#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/e4_tests.log
[ $rc -le 1 ] || exit $rc
U=spittle_amd/ubench; T="timeout -k 5 60"
{
for v in "1 1 0" "1 0 0" "1 0 1" "2 1 0" "2 0 1" "4 0 1" "8 0 1" "8 1 0" "4 1 0"; do set -- $v; $T $U xattn 8 1500 $1 1 1 $2 $3; done
for np in 0 2 4; do $T $U gemv 5120 1280 8 1 1 1 1 $np; done
$T $U gemv 5120 1280 8 2 0 1
for np in 0 2 4; do $T $U gemv 3840 1280 8 3 1 1 1 $np; done
$T $U layer 8 1 2 - 2 2 4 1
$T $U layer 8 1 1 - 2 2 4 1
$T $U layer 8 1 2 - 2 2 4 0
$T $U layer 8 1 4 - 2 2 4 1
$T $U layer 8 1 8 - 2 2 4 1
$T $U layer 8 1 2 - 4 4 4 1
} > gpurun_out/e4_ubench.log 2>&1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e4_bench.log 2>&1; tail -1 gpurun_out/e4_bench.log
