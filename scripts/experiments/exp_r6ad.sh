#!/bin/bash
# r6ad: exact 12-wave split as the default for C2's direct GEMVs: the whole -m gpu suite and the C2 line.
bash scripts/gpu_steps.sh \
  "r6ad_tests|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6ad_c2|200|python3 scripts/c2_decode_ab.py"
