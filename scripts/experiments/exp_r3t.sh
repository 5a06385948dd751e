#!/bin/bash
# GPU box: fixed vs per-k-step cost of the 128 x 128 (and 256 x 256) tile at the Parakeet streaming
# shape (M = 832): K swept 64 .. 2048 for the SiLU (5), bias (0) and split-K partial (8) epilogues
cd "$GRAFT_REPO_ROOT" || exit 1
U=spittle_amd/ubench
for epi in 5 0 8; do for K in 64 128 256 512 1024 2048; do
  timeout -k 5 60 $U gemm 832 4096 $K $epi 2 || exit 1
done; done
for K in 64 256 1024; do timeout -k 5 60 $U gemm 832 1024 $K 8 2 || exit 1; done
