#!/bin/bash
# r6n: the residual GEMMs (out-proj, fc2) on the 128 x 128 tile with two workgroups per CU
# (SPT_GEMM_RESID128 = 1: out-proj only, 2: both) against the 256 x 256 tile; A/B alternating,
# then per-kernel stats with one window group.
P="python3 scripts/enc_ab.py ."
bash scripts/gpu_steps.sh \
  "r6n_r0|200|SPT_GEMM_RESID128=0 $P" \
  "r6n_r1|200|SPT_GEMM_RESID128=1 $P" \
  "r6n_r2|200|SPT_GEMM_RESID128=2 $P" \
  "r6n_r0b|200|SPT_GEMM_RESID128=0 $P" \
  "r6n_r1b|200|SPT_GEMM_RESID128=1 $P" \
  "r6n_r2b|200|SPT_GEMM_RESID128=2 $P" \
  "r6n_g1_r0|200|SPT_ENC_GROUPS=1 SPT_GEMM_RESID128=0 $P" \
  "r6n_g1_r1|200|SPT_ENC_GROUPS=1 SPT_GEMM_RESID128=1 $P" \
  "r6n_prof_r1|300|SPT_ENC_GROUPS=1 SPT_GEMM_RESID128=2 rocprofv3 --kernel-trace --stats -d gpurun_out/r6n_prof_r1 -o prof -- python3 scripts/enc_ab.py ." \
  "r6n_prof_top|120|python3 scripts/rocpd_top.py gpurun_out/r6n_prof_r1/prof_results.db 20 && rm -rf gpurun_out/r6n_prof_r1"
