#!/bin/bash
U=spittle_amd/ubench; T="timeout -k 5 60"
{
$T $U gemm 4096 4096 4096 0 1
$T $U gemm 12000 3840 1280 0 1
$T $U gemm 12000 5120 1280 1 1
$T $U gemm 12000 1280 5120 3 1
$T $U gemm 12000 1280 5120 0 1
$T $U gemm 12000 1280 1280 0 1
$T $U gemm 12000 81920 1280 4 1
$T $U gemm 12000 1280 3840 2 1
$T $U gemm 1000 1280 1280 0 1
} > gpurun_out/e7_gemm.log 2>&1; cat gpurun_out/e7_gemm.log
