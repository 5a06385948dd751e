# round 5: encoder window groups on concurrent streams (SPT_ENC_GROUPS): bitwise test, then the
# bench's encoder_ms per grouping
bash scripts/gpu_steps.sh \
 "r5t_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'groups_bitwise'" \
 "r5t_g1|300|SPT_ENC_GROUPS=1 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5t_g2|300|SPT_ENC_GROUPS=2 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5t_g3|300|SPT_ENC_GROUPS=3 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5t_g4|300|SPT_ENC_GROUPS=4 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5t_g2e|300|SPT_ENC_GRAPH=0 SPT_ENC_GROUPS=2 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
