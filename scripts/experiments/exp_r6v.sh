#!/bin/bash
# r6v: (a) the finalize kernel's done flag and position row fetched up front (bitwise) and (b) the
# decoder self-attention in 4-wave workgroups (SPT_SA_NW=4) against the previous build, alternating,
# B = 8 and 1; outputs compared bitwise.
O="B1_PKG=scratch_ab/r6base"
bash scripts/gpu_steps.sh \
  "r6v_b8_old|200|$O B1_DUMP=gpurun_out/r6v_b8_old.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b8_new|200|B1_DUMP=gpurun_out/r6v_b8_new.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b8_nw4|200|SPT_SA_NW=4 B1_DUMP=gpurun_out/r6v_b8_nw4.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b8_oldb|200|$O B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b8_newb|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b8_nw4b|200|SPT_SA_NW=4 B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6v_b1_old|200|$O python3 scripts/probe_b1.py" \
  "r6v_b1_new|200|python3 scripts/probe_b1.py" \
  "r6v_b1_nw4|200|SPT_SA_NW=4 python3 scripts/probe_b1.py" \
  "r6v_b1_oldb|200|$O python3 scripts/probe_b1.py" \
  "r6v_b1_newb|200|python3 scripts/probe_b1.py" \
  "r6v_b1_nw4b|200|SPT_SA_NW=4 python3 scripts/probe_b1.py" \
  "r6v_cmp|60|python3 -c \"import numpy as np
x = np.load('gpurun_out/r6v_b8_old.npz')
for n in ('new', 'nw4'):
    y = np.load('gpurun_out/r6v_b8_%s.npz' % n)
    print(n, {k: bool(np.array_equal(x[k], y[k])) for k in ('tokens', 'top1', 'top2')}, float(np.abs(x['top1'] - y['top1']).max()))\""
