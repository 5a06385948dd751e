# r4a: encoder attention SUM=4 (Q pre-scaled by log2(e)/8, the score accumulator starts at -m, one
# v_exp + one scalar add per score) against SUM=3 (r3 default): probe time + whole encoder, then
# the encoder parity tests and the full-size tests under SUM=4
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 3 4 3 4; do
  SPT_ATTN_SUM=$v timeout -k 10 300 python -u scripts/probe_kernels.py enc_attn enc_fc1_gemm > gpurun_out/r4a_probe_$v.log 2>&1 || { tail -5 gpurun_out/r4a_probe_$v.log; exit 1; }
  echo "SUM=$v $(tail -1 gpurun_out/r4a_probe_$v.log)"
done
SPT_ATTN_SUM=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { tail -20 gpurun_out/r4a_tests.log; exit 1; }
tail -1 gpurun_out/r4a_tests.log
