# round 5: encoder attention V-tile swizzle (SPT_ATTN_SWZ=3) against the default, in-sequence probe; bitwise check of the encoder output
bash scripts/gpu_steps.sh \
 "r5q_a1|200|python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm" \
 "r5q_a3|200|SPT_ATTN_SWZ=3 python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm" \
 "r5q_a1b|200|python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm" \
 "r5q_a3b|200|SPT_ATTN_SWZ=3 python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm" \
 "r5q_eq|300|python3 -u scripts/enc_swz_bitwise.py"
