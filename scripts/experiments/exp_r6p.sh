#!/bin/bash
# r6p: the head's final LayerNorm once (dec_final_ln) and the logits GEMV on the staged rows
# (SPT_LOGITS_LN=1) instead of every one of its 811 workgroups staging the LayerNorm of x + the
# pending slabs itself.  Decode pass at B = 8 / 1, alternating; tokens / top-1 / top-2 compared
# bitwise between the two.
bash scripts/gpu_steps.sh \
  "r6p_b8_0|200|B1_DUMP=gpurun_out/r6p_b8_0.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6p_b8_1|200|SPT_LOGITS_LN=1 B1_DUMP=gpurun_out/r6p_b8_1.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6p_b8_0b|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6p_b8_1b|200|SPT_LOGITS_LN=1 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6p_b1_0|200|B1_DUMP=gpurun_out/r6p_b1_0.npz python3 scripts/probe_b1.py" \
  "r6p_b1_1|200|SPT_LOGITS_LN=1 B1_DUMP=gpurun_out/r6p_b1_1.npz python3 scripts/probe_b1.py" \
  "r6p_b1_0b|200|python3 scripts/probe_b1.py" \
  "r6p_b1_1b|200|SPT_LOGITS_LN=1 python3 scripts/probe_b1.py" \
  "r6p_cmp|60|python3 -c \"import numpy as np
for b in ('b8', 'b1'):
    x, y = np.load('gpurun_out/r6p_%s_0.npz' % b), np.load('gpurun_out/r6p_%s_1.npz' % b)
    print(b, {k: bool(np.array_equal(x[k], y[k])) for k in ('tokens', 'top1', 'top2')})\""
