#!/bin/bash
# r6ag: C2 logits GEMV (f32, K = 12 super-steps) with each wave's exact K slice in flight (SPT_GV_LOGITS_KS=1:
# 8 waves, 2 column tiles, K over 4 waves) against the default (4 waves x 4 tiles, 3 dependent chunks).
C="python3 scripts/c2_decode_ab.py"
bash scripts/gpu_steps.sh "r6ag_0|200|$C" "r6ag_1|200|SPT_GV_LOGITS_KS=1 $C" "r6ag_0b|200|$C" "r6ag_1b|200|SPT_GV_LOGITS_KS=1 $C"
