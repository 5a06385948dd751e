#!/bin/bash
# r6w: Whisper-small f32 at B = 1 (C2) with its encoder GEMMs on the 64-row tiles (SPT_GEMM_F32_SMALL=1:
# 72-288 128 x 128 tiles left most of the 256 CUs idle) against the 128 x 128 tile, alternating;
# then the f32 parity tests with it on.
P="ENC_AB_B=1 ENC_AB_DTYPE=f32 ENC_AB_MODEL=synthetic:small python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6w_0|200|$P" \
  "r6w_1|200|SPT_GEMM_F32_SMALL=1 $P" \
  "r6w_0b|200|$P" \
  "r6w_1b|200|SPT_GEMM_F32_SMALL=1 $P" \
  "r6w_tests|600|SPT_GEMM_F32_SMALL=1 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread"
