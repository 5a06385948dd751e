# r2 session 3: cross-attention key split (merged by the cross-out GEMV's A_ATTN prologue) re-measured on the current decoder
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_m.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_m.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run SPT_XATTN_SPLIT=1
run SPT_XATTN_SPLIT=2
run SPT_XATTN_SPLIT=3
