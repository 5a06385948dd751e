# round 5: 32- vs 64-query attention inside the bench's encoder (alternating, with and without the
# window groups)
B="python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
bash scripts/gpu_steps.sh \
 "r5ah_q1a|300|$B" "r5ah_q0a|300|SPT_ATTN_Q32S=0 $B" \
 "r5ah_q1b|300|$B" "r5ah_q0b|300|SPT_ATTN_Q32S=0 $B" \
 "r5ah_q1c|300|$B" "r5ah_q0c|300|SPT_ATTN_Q32S=0 $B" \
 "r5ah_g1q1|300|SPT_ENC_GROUPS=1 $B" "r5ah_g1q0|300|SPT_ENC_GROUPS=1 SPT_ATTN_Q32S=0 $B"
