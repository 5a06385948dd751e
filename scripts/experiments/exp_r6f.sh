#!/bin/bash
# r6f: the LayerNorm fold with FMA epilogues (A/B on one box, alternating); the persistent pass with
# its layer table in LDS (chain vs persistent at B = 1 / 8, stamps); the persistent + parity tests.
P="python3 scripts/enc_ab.py"
bash scripts/gpu_steps.sh \
  "r6f_nofold|200|SPT_LN_FOLD=0 $P ." \
  "r6f_fold|200|$P ." \
  "r6f_nofold2|200|SPT_LN_FOLD=0 $P ." \
  "r6f_fold2|200|$P ." \
  "r6f_pd_b1_chain|200|python3 scripts/probe_b1.py" \
  "r6f_pd_b1|200|SPT_PERSISTENT=1 python3 scripts/probe_b1.py" \
  "r6f_pd_b8_chain|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6f_pd_b8|200|SPT_PERSISTENT=1 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6f_pd_b1_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1_r6f.bin python3 scripts/probe_b1.py" \
  "r6f_tests|600|python3 -u -m pytest tests/test_gpu_persistent.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread"
