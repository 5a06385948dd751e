#!/bin/bash
# r6al: fc2's residual fold into slab 0 (SPT_DEC_XFOLD): bitwise tests, then alternating bench lines
# (C3 + C2 decode) with the fold off / on.
Q="--no-parakeet --no-turbo --no-app-latency --no-cpu-baseline --no-probe"
bash scripts/gpu_steps.sh \
  "r6al_tests|600|python3 -u -m pytest tests/test_gpu_full.py tests/test_gpu_full_large.py -m gpu -x -q -k fold --timeout 300 --timeout-method thread" \
  "r6al_b0a|400|SPT_DEC_XFOLD=0 python3 bench.py $Q" \
  "r6al_b1a|400|SPT_DEC_XFOLD=1 python3 bench.py $Q" \
  "r6al_b0b|400|SPT_DEC_XFOLD=0 python3 bench.py $Q" \
  "r6al_b1b|400|SPT_DEC_XFOLD=1 python3 bench.py $Q"
