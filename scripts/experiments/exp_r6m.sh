#!/bin/bash
# r6m: de-synchronised first round of the 256x256 GEMM (SPT_G2_DESYNC = start delay of every other
# first-round workgroup per XCD, in 8128-cycle units): do the epilogue store bursts of lock-step CUs
# cost encoder time?  A/B alternating, default two window groups and one group.
P="python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6m_d0|200|SPT_G2_DESYNC=0 $P" \
  "r6m_d1|200|SPT_G2_DESYNC=1 $P" \
  "r6m_d2|200|SPT_G2_DESYNC=2 $P" \
  "r6m_d4|200|SPT_G2_DESYNC=4 $P" \
  "r6m_d0b|200|SPT_G2_DESYNC=0 $P" \
  "r6m_d2b|200|SPT_G2_DESYNC=2 $P" \
  "r6m_g1_d0|200|SPT_ENC_GROUPS=1 SPT_G2_DESYNC=0 $P" \
  "r6m_g1_d2|200|SPT_ENC_GROUPS=1 SPT_G2_DESYNC=2 $P" \
  "r6m_g1_d4|200|SPT_ENC_GROUPS=1 SPT_G2_DESYNC=4 $P" \
  "r6m_g1_d0b|200|SPT_ENC_GROUPS=1 SPT_G2_DESYNC=0 $P"
