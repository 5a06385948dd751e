#!/bin/bash
# r6d: encoder A/B on one box -- r5 build vs this tree (fold off / on), each under one window group
# and the default two; per-kernel rocprofv3 stats, one group, fold on / off / r5; then the persistent
# pass after the barrier fix (B = 1 and 8, with and without stamps) against the launch chain.
P="python3 scripts/enc_ab.py"
bash scripts/gpu_steps.sh \
  "r6d_r5|200|$P scratch_ab/r5" \
  "r6d_nofold|200|SPT_LN_FOLD=0 $P ." \
  "r6d_fold|200|$P ." \
  "r6d_r5_g1|200|SPT_ENC_GROUPS=1 $P scratch_ab/r5" \
  "r6d_nofold_g1|200|SPT_ENC_GROUPS=1 SPT_LN_FOLD=0 $P ." \
  "r6d_fold_g1|200|SPT_ENC_GROUPS=1 $P ." \
  "r6d_r5_again|200|$P scratch_ab/r5" \
  "r6d_pd_b1_chain|200|python3 scripts/probe_b1.py" \
  "r6d_pd_b1|200|SPT_PERSISTENT=1 python3 scripts/probe_b1.py" \
  "r6d_pd_b8_chain|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6d_pd_b8|200|SPT_PERSISTENT=1 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6d_pd_b1_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1_r6d.bin python3 scripts/probe_b1.py" \
  "r6d_pd_b8_stamp|200|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b8_r6d.bin B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6d_prof_fold|300|SPT_ENC_GROUPS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_fold -o prof -- python3 scripts/enc_ab.py ." \
  "r6d_prof_nofold|300|SPT_ENC_GROUPS=1 SPT_LN_FOLD=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_nofold -o prof -- python3 scripts/enc_ab.py ." \
  "r6d_prof_r5|300|SPT_ENC_GROUPS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_r5 -o prof -- python3 scripts/enc_ab.py scratch_ab/r5"
