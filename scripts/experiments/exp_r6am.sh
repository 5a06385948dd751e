#!/bin/bash
# r6am: with the residual fold (two slab rows per LayerNorm prologue), re-try the wider workgroups
# that read them: logits 8 column tiles per workgroup (SPT_GV_LOGITS_CT=8), QKV two column tiles
# (SPT_GV_CT2_MIN=3840); alternating with the default.
Q="--no-parakeet --no-turbo --no-app-latency --no-cpu-baseline --no-probe"
bash scripts/gpu_steps.sh \
  "r6am_base_a|400|python3 bench.py $Q" \
  "r6am_lct8|400|SPT_GV_LOGITS_CT=8 python3 bench.py $Q" \
  "r6am_ct2|400|SPT_GV_CT2_MIN=3840 python3 bench.py $Q" \
  "r6am_base_b|400|python3 bench.py $Q" \
  "r6am_lct8_b|400|SPT_GV_LOGITS_CT=8 python3 bench.py $Q" \
  "r6am_ct2_b|400|SPT_GV_CT2_MIN=3840 python3 bench.py $Q"
