#!/bin/bash
# r6q: decoder cross-attention knobs re-measured on the round-6 tree at B = 8 (the C3 decode): key
# blocks in flight per wave (SPT_XATTN_PF 2 / 3 / 4) and key chunks merged by the cross output
# projection's prologue (SPT_XATTN_SPLIT 2 / 4), against the default, alternating.
P="B1_BATCH=8 python3 scripts/probe_b1.py"
bash scripts/gpu_steps.sh \
  "r6q_def|200|$P" \
  "r6q_pf3|200|SPT_XATTN_PF=3 $P" \
  "r6q_pf4|200|SPT_XATTN_PF=4 $P" \
  "r6q_sp2|200|SPT_XATTN_SPLIT=2 $P" \
  "r6q_sp4|200|SPT_XATTN_SPLIT=4 $P" \
  "r6q_def2|200|$P" \
  "r6q_pf3b|200|SPT_XATTN_PF=3 $P" \
  "r6q_sp2b|200|SPT_XATTN_SPLIT=2 $P"
