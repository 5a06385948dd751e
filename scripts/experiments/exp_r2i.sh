# r2 session 3: decoder row limit (auto decode groups) -- batching tests, full -m gpu suite, bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batching.py -x -v --timeout 200 --timeout-method thread > gpurun_out/batching.log 2>&1
rc=$?; tail -8 gpurun_out/batching.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_s3b.log 2>&1
rc=$?; tail -4 gpurun_out/tests_s3b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_s3b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_s3b.log; exit 1; }
tail -1 gpurun_out/bench_s3b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])'
