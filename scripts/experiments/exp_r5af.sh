# round 5: encoder attention with 32 queries per wave and three workgroups per CU
# (SPT_ATTN_Q32S=1, bitwise the default): bitwise test, repeatability, probes A/B, bench A/B
bash scripts/gpu_steps.sh \
 "r5af_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'schedules'" \
 "r5af_rep|400|SPT_ATTN_Q32S=1 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k 'repeatable'" \
 "r5af_a0|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5af_a1|200|SPT_ATTN_Q32S=1 python3 scripts/probe_kernels.py enc_attn" \
 "r5af_a0b|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5af_a1b|200|SPT_ATTN_Q32S=1 python3 scripts/probe_kernels.py enc_attn" \
 "r5af_b1|300|SPT_ATTN_Q32S=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5af_b0|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
