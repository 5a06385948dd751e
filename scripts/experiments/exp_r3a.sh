# r3: K split of the decoder's self-/cross-attention output projections into pending slabs
# (summed by the next LayerNorm prologue): 80 -> 160 / 320 workgroups per launch
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_r3a.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_r3a.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_r3a.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run SPT_SO_SPLIT=1
run SPT_SO_SPLIT=2
run SPT_SO_SPLIT=4
run SPT_CO_SPLIT=2
run SPT_CO_SPLIT=4
run SPT_SO_SPLIT=4 SPT_CO_SPLIT=4
run SPT_SO_SPLIT=2 SPT_CO_SPLIT=2
run SPT_SO_SPLIT=1
