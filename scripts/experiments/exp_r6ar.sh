#!/bin/bash
# r6ar: Parakeet decode read-backs into pinned memory, output rows trimmed to the longest emitted
# row: Parakeet GPU tests, then two Parakeet bench lines (compare r6aq).
bash scripts/gpu_steps.sh \
  "r6ar_tests|600|python3 -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6ar_p1a|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ar_p1b|300|python3 bench.py --parakeet-only --no-cpu-baseline"
