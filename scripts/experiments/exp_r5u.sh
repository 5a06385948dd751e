# round 5: Parakeet encoder window groups on concurrent streams (SPT_PK_GROUPS): bitwise tests,
# then the C5 lines per grouping
bash scripts/gpu_steps.sh \
 "r5u_par|400|python -u -m pytest tests/test_gpu_parakeet.py -m gpu -v --timeout 200 --timeout-method thread -k 'groups_bitwise or c5_streaming or bitwise_invariant'" \
 "r5u_g1|300|SPT_PK_GROUPS=1 python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5u_g2|300|SPT_PK_GROUPS=2 python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5u_g4|300|SPT_PK_GROUPS=4 python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5u_g3|300|SPT_PK_GROUPS=3 python -u bench.py --parakeet-only --no-cpu-baseline"
