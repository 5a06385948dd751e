#!/bin/bash
# r6ae: B = 1 knobs on the round-6 tree: cross-attention ring depth (SPT_XATTN_PF 3 / 4; at B = 1 the
# single-wave vw kernel streams each head's window with 96-160 waves) and the logits GEMV with 8 column
# tiles per workgroup (SPT_GV_LOGITS_CT=8), for C2 (small f32) and large-v3 bf16; alternating.
C="python3 scripts/c2_decode_ab.py"
L="python3 scripts/probe_b1.py"
bash scripts/gpu_steps.sh \
  "r6ae_c2_def|200|$C" "r6ae_c2_pf3|200|SPT_XATTN_PF=3 $C" "r6ae_c2_pf4|200|SPT_XATTN_PF=4 $C" "r6ae_c2_ct8|200|SPT_GV_LOGITS_CT=8 $C" \
  "r6ae_c2_defb|200|$C" "r6ae_c2_pf3b|200|SPT_XATTN_PF=3 $C" "r6ae_c2_pf4b|200|SPT_XATTN_PF=4 $C" "r6ae_c2_ct8b|200|SPT_GV_LOGITS_CT=8 $C" \
  "r6ae_l_def|200|$L" "r6ae_l_pf3|200|SPT_XATTN_PF=3 $L" "r6ae_l_pf4|200|SPT_XATTN_PF=4 $L" "r6ae_l_ct8|200|SPT_GV_LOGITS_CT=8 $L" \
  "r6ae_l_defb|200|$L" "r6ae_l_pf3b|200|SPT_XATTN_PF=3 $L" "r6ae_l_pf4b|200|SPT_XATTN_PF=4 $L" "r6ae_l_ct8b|200|SPT_GV_LOGITS_CT=8 $L"
