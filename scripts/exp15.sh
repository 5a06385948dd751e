#!/bin/bash
# r1 exp15: self-out / fc2 K splits (1 = residual update in the projection, no pending slabs)
cd spittle_amd
for i in 1 2; do for so in 2 1; do for fs in 2 1; do
  SOS=$so FC2S=$fs timeout -k 5 60 ./ubench layer 8 1 > /tmp/o.txt || exit 1; sed "s/^/so=$so fc2=$fs /" /tmp/o.txt
done; done; done
