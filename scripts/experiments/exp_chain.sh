#!/bin/bash
# decoder GEMV chains (graph, cache-cold): per-launch time and the workgroup timeline; PMC passes
mkdir -p gpurun_out; cd spittle_amd
for k in 0 1 2 3 4 5; do
  for G in 80 160 256; do
    if [ $k -ne 0 ] && [ $G -ne 80 ]; then continue; fi
    timeout -k 5 60 ./ubench_stamp chain $k 48 $G || exit 1
    timeout -k 5 60 ./ubench chain $k 48 $G || exit 1
  done
done
cd .. && bash scripts/pmc.sh r2 && python3 scripts/pmc_parse.py r2
