#!/bin/bash
# r6z: the f32 encoder attention in 2-wave workgroups (64 queries: 288 workgroups for one 30 s window of
# Whisper-small instead of 144) against 4-wave ones (SPT_ATTN_F32_NW=4), C2 shape; encoder output bitwise
# compared; then the f32 test suites.
P="ENC_AB_B=1 ENC_AB_DTYPE=f32 ENC_AB_MODEL=synthetic:small python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6z_nw4|200|SPT_ATTN_F32_NW=4 $P" \
  "r6z_nw2|200|$P" \
  "r6z_nw4b|200|SPT_ATTN_F32_NW=4 $P" \
  "r6z_nw2b|200|$P" \
  "r6z_dump4|200|SPT_ATTN_F32_NW=4 python3 scripts/enc_dump.py synthetic:small f32 gpurun_out/r6z_4.npz" \
  "r6z_dump2|200|python3 scripts/enc_dump.py synthetic:small f32 gpurun_out/r6z_2.npz" \
  "r6z_cmp|60|python3 -c \"import numpy as np; a = np.load('gpurun_out/r6z_4.npz')['enc']; b = np.load('gpurun_out/r6z_2.npz')['enc']; print('bitwise', bool(np.array_equal(a, b)), float(np.abs(a - b).max()))\"" \
  "r6z_tests|600|python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread"
