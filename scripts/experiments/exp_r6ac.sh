#!/bin/bash
# r6ac: C2 decoder self-out / cross-out (A_DIRECT / attention merge, 12 f32 super-steps) on the exact 12-wave
# split too (SPT_GV_EXACT12_DIRECT=1), against the default, alternating.
bash scripts/gpu_steps.sh \
  "r6ac_0|200|python3 scripts/c2_decode_ab.py" \
  "r6ac_1|200|SPT_GV_EXACT12_DIRECT=1 python3 scripts/c2_decode_ab.py" \
  "r6ac_0b|200|python3 scripts/c2_decode_ab.py" \
  "r6ac_1b|200|SPT_GV_EXACT12_DIRECT=1 python3 scripts/c2_decode_ab.py"
