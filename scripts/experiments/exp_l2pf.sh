# r2 exp: decoder successor-weight L2 prefetch edges (SPT_L2PF bitmask), bench A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 31 63 15 0 31; do
  SPT_L2PF=$m timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-parakeet > gpurun_out/bench_l2pf$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/bench_l2pf$m.log; exit 1; }
  echo "l2pf=$m $(tail -1 gpurun_out/bench_l2pf$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"], {k: round(v["avg_us"],2) for k,v in d["kernels"].items()})')"
done
