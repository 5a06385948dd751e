#!/bin/bash
# r1 exp13: logits GEMV (LN prologue over x + 4 pending slabs) with / without the register prefetch of the rows
cd spittle_amd
for v in ubench ubench_nopref; do
  for i in 1 2; do
    timeout -k 5 60 ./$v gemv 51866 1280 8 4 1 1 1 4 | sed "s/^/$v /" || exit 1
  done
done
