#!/bin/bash
# r6aq: Parakeet mirror's cheaper ctypes conversions (result arrays via string_at, one cast of the
# PCM pointer array): Parakeet GPU tests, then two Parakeet bench lines (compare r6ap's p1 lines).
bash scripts/gpu_steps.sh \
  "r6aq_tests|600|python3 -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6aq_p1a|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6aq_p1b|300|python3 bench.py --parakeet-only --no-cpu-baseline"
