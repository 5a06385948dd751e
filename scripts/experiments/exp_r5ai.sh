# round 5: encoder window groupings other than the default across the parity / full-size / whisper_full suites
bash scripts/gpu_steps.sh \
 "r5ai_g1|600|SPT_ENC_GROUPS=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r5ai_g4|600|SPT_ENC_GROUPS=4 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_full.py -m gpu -x -q --timeout 300 --timeout-method thread"
