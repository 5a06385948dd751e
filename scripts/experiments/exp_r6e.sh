#!/bin/bash
# r6e: the LayerNorm fold with DPP butterflies and preloaded row statistics (A/B on one box), the
# persistent pass's stamps with the compute-side barrier-B split, then the persistent tests.
P="python3 scripts/enc_ab.py"
bash scripts/gpu_steps.sh \
  "r6e_nofold|200|SPT_LN_FOLD=0 $P ." \
  "r6e_fold|200|$P ." \
  "r6e_nofold2|200|SPT_LN_FOLD=0 $P ." \
  "r6e_fold2|200|$P ." \
  "r6e_prof_fold|300|SPT_ENC_GROUPS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_prof_fold -o prof -- python3 scripts/enc_ab.py ." \
  "r6e_pd_b1_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1_r6e.bin python3 scripts/probe_b1.py" \
  "r6e_tests|600|python3 -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread"
