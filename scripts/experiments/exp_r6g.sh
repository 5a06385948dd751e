#!/bin/bash
# r6g: the persistent pass with constant-index kernel arguments (no scratch), global-qualified table
# pointers and unconditional prefetch loads: chain vs persistent at B = 1 / 8, stamps, tests.
bash scripts/gpu_steps.sh \
  "r6g_pd_b1_chain|200|python3 scripts/probe_b1.py" \
  "r6g_pd_b1|200|SPT_PERSISTENT=1 python3 scripts/probe_b1.py" \
  "r6g_pd_b8_chain|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6g_pd_b8|200|SPT_PERSISTENT=1 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6g_pd_b1_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1_r6g.bin python3 scripts/probe_b1.py" \
  "r6g_pd_b8_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b8_r6g.bin B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6g_tests|600|python3 -u -m pytest tests/test_gpu_persistent.py -m gpu -x -q --timeout 300 --timeout-method thread"
