# round 5: encoder attention with Q in LDS (no spills) A/B, parity
bash scripts/gpu_steps.sh \
 "r5f_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread" \
 "r5f_b1|300|python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo" \
 "r5f_b0|300|SPT_ATTN_QL=0 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo"
