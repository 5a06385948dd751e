#!/bin/bash
# r6j: LayerNorm fold with last-arriver row statistics (the producers' last column tile of each row
# block merges the partials; consumers read {mean, rstd}): parity + A/B + per-kernel stats.
P="python3 scripts/enc_ab.py"
bash scripts/gpu_steps.sh \
  "r6j_tests|600|python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6j_nofold|200|SPT_LN_FOLD=0 $P ." \
  "r6j_fold|200|$P ." \
  "r6j_nofold2|200|SPT_LN_FOLD=0 $P ." \
  "r6j_fold2|200|$P ." \
  "r6j_prof_fold|300|SPT_ENC_GROUPS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6j_prof_fold -o prof -- python3 scripts/enc_ab.py ."
