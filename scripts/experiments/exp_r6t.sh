#!/bin/bash
# r6t: relaxed arrival counters in the decode-step finalize kernels (no L2 write-back / invalidate in every block's tail) against
# the previous build (scratch_ab/r6base), alternating, B = 8 and 1; outputs compared bitwise; then the decoder suites.
bash scripts/gpu_steps.sh \
  "r6t_b8_old|200|B1_PKG=scratch_ab/r6base B1_DUMP=gpurun_out/r6t_b8_old.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6t_b8_new|200|B1_DUMP=gpurun_out/r6t_b8_new.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6t_b8_oldb|200|B1_PKG=scratch_ab/r6base B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6t_b8_newb|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6t_b1_old|200|B1_PKG=scratch_ab/r6base B1_DUMP=gpurun_out/r6t_b1_old.npz python3 scripts/probe_b1.py" \
  "r6t_b1_new|200|B1_DUMP=gpurun_out/r6t_b1_new.npz python3 scripts/probe_b1.py" \
  "r6t_b1_oldb|200|B1_PKG=scratch_ab/r6base python3 scripts/probe_b1.py" \
  "r6t_b1_newb|200|python3 scripts/probe_b1.py" \
  "r6t_cmp|60|python3 -c \"import numpy as np
for b in ('b8', 'b1'):
    x, y = np.load('gpurun_out/r6t_%s_old.npz' % b), np.load('gpurun_out/r6t_%s_new.npz' % b)
    print(b, {k: bool(np.array_equal(x[k], y[k])) for k in ('tokens', 'top1', 'top2')})\"" \
  "r6t_tests|700|python3 -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py tests/test_gpu_full_large.py -m gpu -x -q --timeout 300 --timeout-method thread"
