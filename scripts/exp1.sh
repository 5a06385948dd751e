#!/bin/bash
# decoder experiments: nt vs default weight loads, cross-attention splits/waves, two-stream overlap
U=spittle_amd/ubench; R=spittle_amd/ubench_ref
T="timeout -k 5 60"
set -e
for b in $U $R; do
  echo "== $b"
  for cfg in "1280 1280 8 2 0" "1280 1280 8 0 1" "3840 1280 8 3 1" "5120 1280 8 1 1" "1280 5120 8 2 0" "51866 1280 8 4 1"; do $T $b gemv $cfg 1; done
  $T $b layer 8 1
done
echo "== attention variants"
for sw in "1 8" "1 16" "2 8" "3 8" "4 8" "2 16" "8 8"; do $T $U attn 8 20 1500 1500 0 1 1 $sw; done
echo "== layer with splits"
for sw in "1 8" "2 8" "4 8" "1 16"; do $T $U layer 8 1 $sw; done
echo "== two streams"
$T $U layer2 4 1
$T $U layer2 8 1
