#!/bin/bash
# HBM traffic of the hot-path kernels from PMC counters (separate passes, no trace domains),
# parsed on the box into profiles/pmc_*.json (the raw CSVs are too large to bring back).
# usage: bash scripts/pmc.sh TAG
TAG=${1:-r2}
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  SPT_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${TAG}_$C -o run -- \
     python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-app-latency --no-probe --no-turbo --no-parakeet --no-c2 --decode-steps 8 \
     > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 scripts/pmc_parse.py ${TAG} > gpurun_out/pmc_${TAG}_parsed.txt && cp profiles/pmc_*.json gpurun_out/ && \
  rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE
