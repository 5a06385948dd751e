# attention optimistic-softmax (SPT_ATTN_SUM=3) A/B: encoder output vs the default kernel, probes, bench, parity
export TMPDIR=/tmp
mkdir -p gpurun_out
SPT_ATTN_SUM=0 timeout -k 10 120 python3 scripts/enc_dump.py s0 > gpurun_out/g6_a.log 2>&1 || { tail -5 gpurun_out/g6_a.log; exit 1; }
SPT_ATTN_SUM=3 timeout -k 10 120 python3 scripts/enc_dump.py s3 > gpurun_out/g6_b.log 2>&1 || { tail -5 gpurun_out/g6_b.log; exit 1; }
tail -1 gpurun_out/g6_a.log; tail -1 gpurun_out/g6_b.log
python3 -c "import numpy as np; a=np.load('gpurun_out/enc_s0.npy'); b=np.load('gpurun_out/enc_s3.npy'); print('rel L2', float(np.linalg.norm(a-b)/np.linalg.norm(a)), 'maxdiff', float(np.abs(a-b).max()))"
for v in 0 3 0 3; do
SPT_ATTN_SUM=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-app-latency --no-parakeet > gpurun_out/g6_bench$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/g6_bench$v.log; exit 1; }
echo "sum=$v $(tail -1 gpurun_out/g6_bench$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["encoder_ms"], d["rooflines"]["encoder"]["frac"], d["kernels"]["enc_attn"]["avg_us"])')"
done
SPT_ATTN_SUM=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g6_tests.log; exit $rc
