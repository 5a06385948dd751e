# round 5: encoder attention as two ping-pong wave groups (SPT_ATTN_PP=1): bitwise against the default
# kernel, repeatability under load, in-sequence probes A/B, bench
bash scripts/gpu_steps.sh \
 "r5w_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'schedules'" \
 "r5w_rep|400|SPT_ATTN_PP=1 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k 'repeatable'" \
 "r5w_a0|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5w_a1|200|SPT_ATTN_PP=1 python3 scripts/probe_kernels.py enc_attn" \
 "r5w_a0b|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5w_a1b|200|SPT_ATTN_PP=1 python3 scripts/probe_kernels.py enc_attn" \
 "r5w_b1|300|SPT_ATTN_PP=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
