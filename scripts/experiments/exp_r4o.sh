# r4o: the encoder attention with its tile loop unrolled by two (constant LDS offsets) and the QK^T
# chains started from a per-query constant: the encoder parity / bitwise tests, then round part B
# (kernel stats of the bench command + PMC passes) on this tree
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -1 gpurun_out/r4o_tests.log
bash scripts/round_b.sh r4
