#!/bin/bash
# r1 exp11: decoder self-attention keys per lane (SPT_SA_NI 0=8, 4, 2) at 4 / 66 / 132 / 260 cached keys
cd spittle_amd
for ni in 0 4 2; do
  for nk in 4 66 132 260; do
    SPT_SA_NI=$ni timeout -k 5 60 ./ubench attn 8 20 448 $nk 1 1 | sed "s/^/ni=$ni /" || exit 1
  done
done
