#!/bin/bash
# r6at: fc2 split 4 ways (SPT_FC2_SPLIT=4: three slab rows left for q/k/v's prologue after the
# residual fold, 320 fc2 workgroups) vs the default 2; alternating bench lines (C3 + C2).
Q="--no-parakeet --no-turbo --no-app-latency --no-cpu-baseline --no-probe"
bash scripts/gpu_steps.sh \
  "r6at_s2a|400|python3 bench.py $Q" \
  "r6at_s4a|400|SPT_FC2_SPLIT=4 python3 bench.py $Q" \
  "r6at_s2b|400|python3 bench.py $Q" \
  "r6at_s4b|400|SPT_FC2_SPLIT=4 python3 bench.py $Q"
