#!/bin/bash
# r6r: Parakeet C5 residual GEMMs' K split capped (SPT_PK_KS_MAX 8 = default / 4 / 2 / 1): every split
# slab is re-read by the next LayerNorm (8 slabs = 27 MB per LayerNorm at M = 832), against the GEMM's
# own parallelism.  bench.py --parakeet-only, alternating.
B="python3 bench.py --parakeet-only --no-cpu-baseline --steps 10 --warmup 3"
bash scripts/gpu_steps.sh \
  "r6r_k8|300|SPT_PK_KS_MAX=8 $B" \
  "r6r_k4|300|SPT_PK_KS_MAX=4 $B" \
  "r6r_k2|300|SPT_PK_KS_MAX=2 $B" \
  "r6r_k1|300|SPT_PK_KS_MAX=1 $B" \
  "r6r_k8b|300|SPT_PK_KS_MAX=8 $B" \
  "r6r_k4b|300|SPT_PK_KS_MAX=4 $B" \
  "r6r_k2b|300|SPT_PK_KS_MAX=2 $B"
