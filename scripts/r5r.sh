# round 5: encoder schedule variants bitwise (parity file), then the final bench line
bash scripts/gpu_steps.sh \
 "r5r_par|300|python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread" \
 "r5r_bench|400|python -u bench.py"
