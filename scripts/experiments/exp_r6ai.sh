#!/bin/bash
# r6ai: bf16 encoder tile thresholds at the app's B = 1 (one 30 s window, M = 1500: q/k/v 360 tiles of 128 x
# 128 = 1.4 rounds, fc1 120 tiles of 256 x 256 = 0.47 rounds) and at C3 (B = 8, two groups of 6000 rows);
# SPT_GEMM_BF16_T256MIN (default 96) / SPT_GEMM_BF16_T128MIN (default 256), alternating.
P1="ENC_AB_B=1 python3 scripts/enc_ab.py ."
P8="python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6ai_b1_def|200|$P1" \
  "r6ai_b1_a|200|SPT_GEMM_BF16_T128MIN=1024 $P1" \
  "r6ai_b1_b|200|SPT_GEMM_BF16_T256MIN=256 $P1" \
  "r6ai_b1_ab|200|SPT_GEMM_BF16_T256MIN=256 SPT_GEMM_BF16_T128MIN=1024 $P1" \
  "r6ai_b1_defb|200|$P1" \
  "r6ai_b1_ab2|200|SPT_GEMM_BF16_T256MIN=256 SPT_GEMM_BF16_T128MIN=1024 $P1" \
  "r6ai_b8_def|200|$P8" \
  "r6ai_b8_a|200|SPT_GEMM_BF16_T128MIN=1024 $P8" \
  "r6ai_b8_b|200|SPT_GEMM_BF16_T256MIN=256 $P8"
