#!/bin/bash
# kernel microbenchmarks on the GPU box
U=spittle_amd/ubench
T="timeout -k 5 60"
$T $U null
for cfg in "1280 1280 8 2 0" "1280 1280 8 0 1" "3840 1280 8 3 1" "5120 1280 8 1 1" "1280 5120 8 2 0" "51866 1280 8 4 1" "1280 1280 32 2 0" "3840 1280 32 3 1"; do $T $U gemv $cfg 1; done
$T $U attn 8 20 1500 1500 0 1 1
$T $U attn 8 20 448 132 1 1 1
$T $U attn 8 20 448 4 1 4 1
$T $U layer 8 1
$T $U gemm 12000 3840 1280 0 1
$T $U gemm 12000 5120 1280 1 1
$T $U gemm 12000 1280 5120 3 1
$T $U gemm 12000 81920 1280 4 1
