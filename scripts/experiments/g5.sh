# staggered 256-tile GEMM A/B: bitwise encoder equality, probes, bench phases, parity tests under the switch
export TMPDIR=/tmp
mkdir -p gpurun_out
SPT_G2_STAGGER=0 timeout -k 10 120 python3 scripts/enc_dump.py base > gpurun_out/g5_a.log 2>&1 || { tail -5 gpurun_out/g5_a.log; exit 1; }
SPT_G2_STAGGER=1 timeout -k 10 120 python3 scripts/enc_dump.py stg > gpurun_out/g5_b.log 2>&1 || { tail -5 gpurun_out/g5_b.log; exit 1; }
tail -1 gpurun_out/g5_a.log; tail -1 gpurun_out/g5_b.log
python3 -c "import numpy as np; a=np.load('gpurun_out/enc_base.npy'); b=np.load('gpurun_out/enc_stg.npy'); print('bitwise equal:', np.array_equal(a,b), 'maxdiff', float(np.abs(a-b).max()))"
for v in 0 1 0 1; do
SPT_G2_STAGGER=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-app-latency --no-parakeet --no-probe > gpurun_out/g5_bench$v.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/g5_bench$v.log; exit 1; }
echo "stg=$v $(tail -1 gpurun_out/g5_bench$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["encoder_ms"], d["phases_ms"]["cross_kv_ms"], d["rooflines"]["encoder"]["frac"])')"
done
SPT_G2_STAGGER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parakeet.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g5_tests.log; exit $rc
