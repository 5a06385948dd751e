#!/bin/bash
# r6aj: group-aware bf16 256-tile threshold (below 128 tiles counted over the window groups that run
# together -> 128 x 128 / 64-row tiles; SPT_GEMM_BF16_T256G=0: the old rule), encoder ms at B = 1 / 4 / 8,
# alternating; encoder output bitwise at B = 1.
P="python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6aj_b1_old|200|SPT_GEMM_BF16_T256G=0 ENC_AB_B=1 $P" "r6aj_b1_new|200|ENC_AB_B=1 $P" \
  "r6aj_b1_oldb|200|SPT_GEMM_BF16_T256G=0 ENC_AB_B=1 $P" "r6aj_b1_newb|200|ENC_AB_B=1 $P" \
  "r6aj_b4_old|200|SPT_GEMM_BF16_T256G=0 ENC_AB_B=4 $P" "r6aj_b4_new|200|ENC_AB_B=4 $P" \
  "r6aj_b4_oldb|200|SPT_GEMM_BF16_T256G=0 ENC_AB_B=4 $P" "r6aj_b4_newb|200|ENC_AB_B=4 $P" \
  "r6aj_b8_old|200|SPT_GEMM_BF16_T256G=0 $P" "r6aj_b8_new|200|$P" \
  "r6aj_dump_old|200|SPT_GEMM_BF16_T256G=0 python3 scripts/enc_dump.py synthetic:large-v3:enc=4:dec=2 bf16 gpurun_out/r6aj_old.npz" \
  "r6aj_dump_new|200|python3 scripts/enc_dump.py synthetic:large-v3:enc=4:dec=2 bf16 gpurun_out/r6aj_new.npz" \
  "r6aj_cmp|60|python3 -c \"import numpy as np; a = np.load('gpurun_out/r6aj_old.npz')['enc']; b = np.load('gpurun_out/r6aj_new.npz')['enc']; print('bitwise', bool(np.array_equal(a, b)), float(np.abs(a - b).max()))\""
