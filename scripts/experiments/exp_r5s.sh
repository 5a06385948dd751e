# round 5: encoder attention V^T reads as inline asm (no compiler vmcnt(0) on the next tile's DMA):
# bitwise against the builtin reads, in-sequence probe A/B, then the bench line
bash scripts/gpu_steps.sh \
 "r5s_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'schedules or encoder_bf16 or drift'" \
 "r5s_a|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5s_a0|200|SPT_ATTN_QL=0 python3 scripts/probe_kernels.py enc_attn" \
 "r5s_a2|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5s_bench|400|python -u bench.py --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo"
