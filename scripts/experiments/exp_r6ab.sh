#!/bin/bash
# r6ab: C2 decoder (Whisper-small f32, B = 1) LayerNorm GEMVs on an exact 12-wave K split (d = 768 = 12
# f32 super-steps: unconditional weight loads, so the LayerNorm overlaps the weight stream) against the
# previous build, alternating; outputs compared (not bitwise: a different cross-wave summation).
O="B1_PKG=scratch_ab/r6base"
bash scripts/gpu_steps.sh \
  "r6ab_old|200|$O B1_DUMP=gpurun_out/r6ab_old.npz python3 scripts/c2_decode_ab.py" \
  "r6ab_new|200|B1_DUMP=gpurun_out/r6ab_new.npz python3 scripts/c2_decode_ab.py" \
  "r6ab_oldb|200|$O python3 scripts/c2_decode_ab.py" \
  "r6ab_newb|200|python3 scripts/c2_decode_ab.py" \
  "r6ab_cmp|60|python3 -c \"import numpy as np; x = np.load('gpurun_out/r6ab_old.npz'); y = np.load('gpurun_out/r6ab_new.npz'); print({k: bool(np.array_equal(x[k], y[k])) for k in ('tokens', 'top1', 'top2')}, float(np.abs(x['top1'] - y['top1']).max()))\"" \
  "r6ab_tests|600|python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread"
