#!/bin/bash
# Encoder MFMA utilisation from PMC counters (north_star: "MFMA utilisation vs gfx950 peak"):
# SQ_VALU_MFMA_BUSY_CYCLES (SIMD-cycles an MFMA occupies; 32 per 32x32x16 bf16) and
# GRBM_GUI_ACTIVE (GPU-busy cycles, summed over the 8 XCDs) per encoder dispatch, one pass with
# the kernel trace for durations.  Parsed on the box into profiles/r2/pmc_encoder_mfma.json.
export TMPDIR=/tmp
mkdir -p gpurun_out
SPT_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
   --output-format csv -d gpurun_out/pmc_mfma -o run -- \
   python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet --decode-steps 8 \
   > gpurun_out/pmc_mfma.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_mfma.log; exit 1; }
python3 scripts/pmc_mfma_parse.py > gpurun_out/pmc_mfma_parsed.txt && cat gpurun_out/pmc_mfma_parsed.txt && \
  cp profiles/r2/pmc_encoder_mfma.json gpurun_out/ && rm -rf gpurun_out/pmc_mfma
