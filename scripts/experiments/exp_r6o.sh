#!/bin/bash
# r6o: fc2 without its K split, the residual added in place (SPT_FC2_SPLIT=0): q/k/v's LayerNorm
# prologue then reads x alone (no pending slabs).  Decode pass at B = 8 / 1 against the default,
# alternating; then the parity tests with it on.
bash scripts/gpu_steps.sh \
  "r6o_b8_s2|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6o_b8_s0|200|SPT_FC2_SPLIT=0 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6o_b8_s2b|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6o_b8_s0b|200|SPT_FC2_SPLIT=0 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6o_b1_s2|200|python3 scripts/probe_b1.py" \
  "r6o_b1_s0|200|SPT_FC2_SPLIT=0 python3 scripts/probe_b1.py" \
  "r6o_b1_s2b|200|python3 scripts/probe_b1.py" \
  "r6o_b1_s0b|200|SPT_FC2_SPLIT=0 python3 scripts/probe_b1.py" \
  "r6o_tests|600|SPT_FC2_SPLIT=0 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread"
