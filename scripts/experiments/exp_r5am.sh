# round 5: decoder A_DIRECT / A_ATTN GEMVs (self-out, cross-out, fc2) on exact 10-wave K slices (SPT_GV_DX=1)
# against the default 8 / 16-wave slices, alternating; then the decoder parity suites under SPT_GV_DX=1
bash scripts/gpu_steps.sh \
 "r5am_d1|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5am_x1|300|SPT_GV_DX=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5am_d2|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5am_x2|300|SPT_GV_DX=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5am_t|600|SPT_GV_DX=1 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread"
