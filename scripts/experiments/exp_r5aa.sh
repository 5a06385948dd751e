# round 5: encoder attention SUM=5 (the -m chain start as an MFMA k-step, no accumulator copies)
# against SUM=4: oracle parity and repeatability with SUM=5, in-sequence probes A/B, bench
bash scripts/gpu_steps.sh \
 "r5aa_par|300|SPT_ATTN_SUM=5 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'encoder_bf16 or drift or transcribe_bf16'" \
 "r5aa_rep|400|SPT_ATTN_SUM=5 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k 'repeatable or encoder'" \
 "r5aa_a4|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5aa_a5|200|SPT_ATTN_SUM=5 python3 scripts/probe_kernels.py enc_attn" \
 "r5aa_a4b|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5aa_a5b|200|SPT_ATTN_SUM=5 python3 scripts/probe_kernels.py enc_attn" \
 "r5aa_b5|300|SPT_ATTN_SUM=5 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5aa_b4|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
