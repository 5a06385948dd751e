#!/bin/bash
# r1 exp16: cross-attention with 2 vs 3 key blocks in flight per wave (8 layers cache-cold; decoder layer)
cd spittle_amd
for i in 1 2; do for v in ubench ubench_nb3; do
  timeout -k 5 60 ./$v xattn 8 1500 1 1 > /tmp/o.txt || exit 1; sed "s/^/$v /" /tmp/o.txt
  timeout -k 5 60 ./$v layer 8 1 > /tmp/o.txt || exit 1; sed "s/^/$v /" /tmp/o.txt
done; done
