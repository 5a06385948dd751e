#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e5_tests.log 2>&1; rc=$?
tail -3 gpurun_out/e5_tests.log
[ $rc -le 1 ] || exit $rc
U=spittle_amd/ubench; T="timeout -k 5 60"
{
$T $U layer 8 1
$T $U gemv 1280 1280 8 0 1 1 1 2
$T $U gemv 1280 1280 8 5 0 1 1 0
$T $U xattn 8 1500 1 1
} > gpurun_out/e5_ubench.log 2>&1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e5_bench.log 2>&1; tail -1 gpurun_out/e5_bench.log | cut -c 1-900
