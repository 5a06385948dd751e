# round 5: encoder attention DMA sources of whole tiles as a row address + fixed lane offsets
# (default) against the clamped per-tile arithmetic (SPT_ATTN_FULLDMA=0): bitwise, probes, bench
bash scripts/gpu_steps.sh \
 "r5ad_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'schedules or encoder_bf16'" \
 "r5ad_a1|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5ad_a0|200|SPT_ATTN_FULLDMA=0 python3 scripts/probe_kernels.py enc_attn" \
 "r5ad_a1b|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5ad_a0b|200|SPT_ATTN_FULLDMA=0 python3 scripts/probe_kernels.py enc_attn" \
 "r5ad_b1|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ad_b0|300|SPT_ATTN_FULLDMA=0 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
