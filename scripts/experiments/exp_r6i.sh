#!/bin/bash
# r6i: where the LayerNorm fold's consumer GEMMs lose time -- SPT_LNF_DBG timing knobs (wrong results):
# 1 no stats merge, 2 no stats in the epilogue, 4 no x o gamma store, 8 no partials store.
P="python3 scripts/enc_ab.py"
bash scripts/gpu_steps.sh \
  "r6i_nofold|200|SPT_LN_FOLD=0 $P ." \
  "r6i_fold|200|$P ." \
  "r6i_dbg1|200|SPT_LNF_DBG=1 $P ." \
  "r6i_dbg3|200|SPT_LNF_DBG=3 $P ." \
  "r6i_dbg12|200|SPT_LNF_DBG=12 $P ." \
  "r6i_dbg15|200|SPT_LNF_DBG=15 $P ." \
  "r6i_nofold2|200|SPT_LN_FOLD=0 $P ." \
  "r6i_fold2|200|$P ." \
  "r6i_prof_dbg3|300|SPT_ENC_GROUPS=1 SPT_LNF_DBG=3 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i_prof_dbg3 -o prof -- python3 scripts/enc_ab.py ." \
  "r6i_prof_fold|300|SPT_ENC_GROUPS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i_prof_fold -o prof -- python3 scripts/enc_ab.py ."
