# r2 session 3: encoder replayed from a per-batch hipGraph (bench A/B, then the -m gpu suite)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_l.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_l.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], d["rooflines"]["encoder"]["frac"])')"
}
run SPT_ENC_GRAPH=0
run SPT_ENC_GRAPH=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_s3c.log 2>&1
rc=$?; tail -4 gpurun_out/tests_s3c.log; exit $rc
