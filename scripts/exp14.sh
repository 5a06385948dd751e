#!/bin/bash
# r1 exp14: fc2 K split 4 vs 2 (pending slabs summed by the next LayerNorm prologue), one decoder layer
cd spittle_amd
for i in 1 2; do for fs in 4 2; do
  FC2S=$fs timeout -k 5 60 ./ubench layer 8 1 | sed "s/^/fc2split=$fs /" || exit 1
done; done
timeout -k 5 60 ./ubench gemv 1280 5120 8 2 0 1 4 | sed "s/^/fc2 ksplit4 /"
timeout -k 5 60 ./ubench gemv 1280 5120 8 2 0 1 2 | sed "s/^/fc2 ksplit2 /"
timeout -k 5 60 ./ubench gemv 3840 1280 8 3 1 1 1 4 | sed "s/^/qkv np4 /"
timeout -k 5 60 ./ubench gemv 3840 1280 8 3 1 1 1 2 | sed "s/^/qkv np2 /"
