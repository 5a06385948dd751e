#!/bin/bash
# r6aa: the f32 64-row-tile threshold (SPT_GEMM_F32_T128MIN: 128 x 128 tiles from this many up; default 256)
# at the C2 shape: fc1 (288 tiles of 128 x 128, 1.125 rounds) on the 64-row tiles at 512 / 1024.
P="ENC_AB_B=1 ENC_AB_DTYPE=f32 ENC_AB_MODEL=synthetic:small python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6aa_256|200|$P" \
  "r6aa_512|200|SPT_GEMM_F32_T128MIN=512 $P" \
  "r6aa_2048|200|SPT_GEMM_F32_T128MIN=2048 $P" \
  "r6aa_256b|200|$P" \
  "r6aa_512b|200|SPT_GEMM_F32_T128MIN=512 $P" \
  "r6aa_2048b|200|SPT_GEMM_F32_T128MIN=2048 $P"
