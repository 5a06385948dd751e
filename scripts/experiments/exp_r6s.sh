#!/bin/bash
# r6s: decoder self-attention with each wave's first key block fetched before the position arrives
# (AttnWave::run_pre) against the previous build (scratch_ab/r6base), alternating, B = 8 and 1;
# outputs compared bitwise (tokens, top-1, top-2); then the decoder parity / bitwise suites.
bash scripts/gpu_steps.sh \
  "r6s_b8_old|200|B1_PKG=scratch_ab/r6base B1_DUMP=gpurun_out/r6s_b8_old.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6s_b8_new|200|B1_DUMP=gpurun_out/r6s_b8_new.npz B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6s_b8_oldb|200|B1_PKG=scratch_ab/r6base B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6s_b8_newb|200|B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6s_b1_old|200|B1_PKG=scratch_ab/r6base B1_DUMP=gpurun_out/r6s_b1_old.npz python3 scripts/probe_b1.py" \
  "r6s_b1_new|200|B1_DUMP=gpurun_out/r6s_b1_new.npz python3 scripts/probe_b1.py" \
  "r6s_b1_oldb|200|B1_PKG=scratch_ab/r6base python3 scripts/probe_b1.py" \
  "r6s_b1_newb|200|python3 scripts/probe_b1.py" \
  "r6s_cmp|60|python3 -c \"import numpy as np
for b in ('b8', 'b1'):
    x, y = np.load('gpurun_out/r6s_%s_old.npz' % b), np.load('gpurun_out/r6s_%s_new.npz' % b)
    print(b, {k: bool(np.array_equal(x[k], y[k])) for k in ('tokens', 'top1', 'top2')})\"" \
  "r6s_tests|700|python3 -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py tests/test_gpu_full_large.py -m gpu -x -q --timeout 300 --timeout-method thread"
