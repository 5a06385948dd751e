#!/bin/bash
# r6ao: Parakeet host PCM through pinned staging + one 2D copy (SPT_PK_PINNED): bitwise tests, then
# alternating Parakeet bench lines with it off / on.
bash scripts/gpu_steps.sh \
  "r6ao_tests|600|python3 -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6ao_p0a|400|SPT_PK_PINNED=0 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ao_p1a|400|SPT_PK_PINNED=1 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ao_p0b|400|SPT_PK_PINNED=0 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ao_p1b|400|SPT_PK_PINNED=1 python3 bench.py --parakeet-only --no-cpu-baseline"
