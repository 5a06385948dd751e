# full -m gpu suite, then a bench line (no CPU baseline) for the encoder / decode phase times
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-parakeet > gpurun_out/g4_bench$i.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/g4_bench$i.log; exit 1; }
tail -1 gpurun_out/g4_bench$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], d["rooflines"]["encoder"]["frac"], {k: round(v["avg_us"],2) for k,v in d["kernels"].items()})'
done
