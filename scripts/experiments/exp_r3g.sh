#!/bin/bash
# GPU box: Parakeet streaming-shape GEMMs (M = 832) through the 128 x 128 tile: LDS ring depth
# (SPT_GEMM_NT_STAGES) x tile raster (SPT_GEMM_NT_RASTER: 0 M-major, 1 N-major)
cd "$GRAFT_REPO_ROOT" || exit 1
U=spittle_amd/ubench
for st in 2 3 4; do for r in 0 1; do
  for cfg in "832 4096 1024 5 2" "832 3072 1024 0 2" "832 1024 1024 8 2 4" "832 1024 4096 8 2 8" "8320 4096 1024 5 2"; do
    SPT_GEMM_NT_RASTER=$r SPT_GEMM_NT_STAGES=$st timeout -k 5 60 $U gemm $cfg | sed "s/^/st=$st r=$r /" || exit 1
  done
done; done
