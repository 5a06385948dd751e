# r3: narrow-column GEMV (one wave per output column, 320 workgroups) for the decoder's self-/cross-
# attention output projections vs the 16-column MFMA tiles (80 workgroups); A/B/A/B on the C3 bench
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_r3b.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_r3b.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_r3b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run SPT_GV_COL=0
run SPT_GV_COL=1
run SPT_GV_COL=0
run SPT_GV_COL=1
