#!/bin/bash
# r1 exp12: cross-attention waves per workgroup at 4 keys per lane (8 layers back to back, cache-cold)
cd spittle_amd
for nw in 8 12 16 162; do
  SPT_XATTN_NW=$nw timeout -k 5 60 ./ubench xattn 8 1500 1 1 | sed "s/^/nw=$nw /" || exit 1
  SPT_XATTN_NW=$nw timeout -k 5 60 ./ubench layer 8 1 | sed "s/^/nw=$nw /" || exit 1
done
