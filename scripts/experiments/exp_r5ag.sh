# round 5: 32-query attention as the default: the whole -m gpu suite, then the bench line
bash scripts/gpu_steps.sh \
 "r5ag_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r5ag_b|400|python -u bench.py --no-cpu-baseline --no-app-latency"
