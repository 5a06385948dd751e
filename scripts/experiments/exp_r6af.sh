#!/bin/bash
# r6af: Parakeet C5 GEMM tile thresholds re-checked on the round-6 tree (SPT_GEMM_T256: the 256 x 256 tile
# from this many workgroups up, default 128; SPT_GEMM_T64=0: no 64-row tiles), bench.py --parakeet-only.
B="python3 bench.py --parakeet-only --no-cpu-baseline --steps 10 --warmup 3"
bash scripts/gpu_steps.sh \
  "r6af_def|300|$B" "r6af_t48|300|SPT_GEMM_T256=48 $B" "r6af_t16|300|SPT_GEMM_T256=16 $B" "r6af_not64|300|SPT_GEMM_T64=0 $B" \
  "r6af_defb|300|$B" "r6af_t48b|300|SPT_GEMM_T256=48 $B"
