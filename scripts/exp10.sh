#!/bin/bash
# r1 exp10: cross-attention waves x keys-per-lane x key splits (8 layers back to back, cache-cold)
cd spittle_amd
for cfg in 8,8 4,8 8,4 4,4; do
  for s in 1 2 3 4; do
    SPT_XATTN_CFG=$cfg timeout -k 5 60 ./ubench xattn 8 1500 $s 1 | sed "s/^/cfg=$cfg /" || exit 1
  done
done
