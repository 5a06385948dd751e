#!/bin/bash
# C2 decode-pass traffic: one rocprofv3 --pmc pass per counter over scripts/c2_probe.py, parsed into
# profiles/r6/pmc_c2_small_f32.json (copied to gpurun_out/ so it comes back).
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/r6
for C in FETCH_SIZE WRITE_SIZE; do
  SPT_NO_GRAPH=1 timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/c2pmc_$C -o run -- \
     python3 scripts/c2_probe.py > gpurun_out/c2pmc_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 scripts/c2_pmc_parse.py gpurun_out/c2pmc && cp profiles/r6/pmc_c2_small_f32.json gpurun_out/ && \
  rm -rf gpurun_out/c2pmc_FETCH_SIZE gpurun_out/c2pmc_WRITE_SIZE
