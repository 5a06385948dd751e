# r2 session 3: fused decode-step QKV + self-attention (bitwise test, bench A/B, then the -m gpu suite)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_qkv.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fused_test.log 2>&1
rc=$?; tail -6 gpurun_out/fused_test.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  SPT_FUSED_QKV=$f timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_fused$f.log 2>&1 || { echo "bench f$f failed"; tail -5 gpurun_out/bench_fused$f.log; exit 1; }
  echo "fused=$f $(tail -1 gpurun_out/bench_fused$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
done
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_s3.log 2>&1
  rc=$?; tail -5 gpurun_out/tests_s3.log; exit $rc
fi
