#!/bin/bash
# r2 exp: unconditional weight loads (LN waits leave the weights in flight) + chunked cross-attention
mkdir -p gpurun_out
cd spittle_amd
for k in 1 2 3 4 5; do timeout -k 5 60 ./ubench_stamp chain $k 48 | grep -A1 chain || exit 1; done
for S in 1 0; do timeout -k 5 60 ./ubench xattn 8 1500 $S || exit 1; done
cd ..
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "not free_running" > gpurun_out/t_r2c.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2c.log; [ $rc -eq 0 ] || exit $rc
for X in 0 1; do
SPT_XATTN_CHUNKED=$X timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --steps 5 > gpurun_out/bench_r2c_$X.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2c_$X.log').read().strip().splitlines()[-1]);print('chunked=$X RTFx',d['value'],d['phases_ms'],d['rooflines']['decode_pass']['ms_per_pass'], d['roofline']['avg_us'])"
done
