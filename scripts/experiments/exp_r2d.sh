#!/bin/bash
# r2 exp: exact 10-wave LayerNorm GEMVs; chunked cross-attention variants; stream ceiling
mkdir -p gpurun_out
cd spittle_amd
for e in 1 0; do for k in 2 3 4; do GV_EXACT_LN=$e timeout -k 5 60 ./ubench_stamp chain $k 48 | sed "s/^/exact=$e /" || exit 1; done; done
for S in 1 0 -1 -2 -3; do timeout -k 5 60 ./ubench xattn 8 1500 $S || exit 1; done
for G in 160 256 512 1024 2048; do timeout -k 5 60 ./ubench stream $G 512 || exit 1; done
timeout -k 5 60 ./ubench stream 1024 256 || exit 1
cd ..
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "not free_running" > gpurun_out/t_r2d.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2d.log; [ $rc -eq 0 ] || exit $rc
for cfg in "GV_EXACT_LN=1 SPT_XATTN_CHUNKED=0" "GV_EXACT_LN=0 SPT_XATTN_CHUNKED=0" "GV_EXACT_LN=1 SPT_XATTN_CHUNKED=1"; do
env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --steps 5 > gpurun_out/bench_r2d.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2d.log').read().strip().splitlines()[-1]);print('$cfg RTFx',d['value'],d['phases_ms']['decode_ms'],d['rooflines']['decode_pass']['ms_per_pass'], d['roofline']['avg_us'])"
done
