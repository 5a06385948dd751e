# r3: the C3 batch (B = 8) decoded as 1 / 2 / 4 concurrent decode groups, each its own graph on
# its own stream (independent latency-bound chains interleave on the GPU)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_r3c.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_r3c.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_r3c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run SPT_DECODE_GROUPS=1
run SPT_DECODE_GROUPS=2
run SPT_DECODE_GROUPS=4
run SPT_DECODE_GROUPS=1
run SPT_DECODE_GROUPS=2
