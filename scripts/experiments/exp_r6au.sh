#!/bin/bash
# r6au: the rebuilt final .so (after reverting the fc2-split experiment): smoke, decoder GPU tests,
# one default bench line.
bash scripts/gpu_steps.sh \
  "r6au_smoke|300|python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r6au_tests|600|python3 -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6au_bench|600|python3 bench.py"
