# round 5: B = 1 app-shape profile (chain and persistent), first without the profiler, then the
# whole -m gpu suite
bash scripts/gpu_steps.sh \
 "r5j_b1plain|200|SPT_PERSISTENT=0 python3 -u scripts/probe_b1.py" \
 "r5j_b1pplain|200|SPT_PERSISTENT=1 python3 -u scripts/probe_b1.py" \
 "r5j_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
