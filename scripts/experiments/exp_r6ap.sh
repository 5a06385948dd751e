#!/bin/bash
# r6ap: Parakeet pinned staging for windows up to 4 s (default) vs per-window pageable copies
# (SPT_PK_PINNED=0): the test, then six alternating Parakeet bench lines.
bash scripts/gpu_steps.sh \
  "r6ap_tests|300|python3 -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q -k pinned --timeout 300 --timeout-method thread" \
  "r6ap_p0a|300|SPT_PK_PINNED=0 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ap_p1a|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ap_p0b|300|SPT_PK_PINNED=0 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ap_p1b|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ap_p0c|300|SPT_PK_PINNED=0 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6ap_p1c|300|python3 bench.py --parakeet-only --no-cpu-baseline"
