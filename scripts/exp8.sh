#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e8_tests.log 2>&1; rc=$?
tail -3 gpurun_out/e8_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 5 60 spittle_amd/ubench gemm 12000 1280 3840 2 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e8_bench.log 2>&1; tail -1 gpurun_out/e8_bench.log | cut -c 1-700
