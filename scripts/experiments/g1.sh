# r2 session 2: encoder-attention variants (probe), decode groups A/B (bench), then the -m gpu suite
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "SPT_ATTN_Q32=1" "SPT_ATTN_SUM=0" "SPT_ATTN_SUM=1" "SPT_ATTN_SUM=2"; do
  env $v timeout -k 10 120 python3 scripts/probe_kernels.py enc_attn enc_fc1_gemm > gpurun_out/probe_$v.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/probe_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/probe_$v.log)"
done
for g in 1 2; do
  SPT_DECODE_GROUPS=$g timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_groups$g.log 2>&1 || { echo "bench g$g failed"; tail -5 gpurun_out/bench_groups$g.log; exit 1; }
  echo "groups=$g $(tail -1 gpurun_out/bench_groups$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"])')"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_s1.log 2>&1
rc=$?; tail -5 gpurun_out/tests_s1.log; exit $rc
