#!/bin/bash
# r2 exp: GEMV operand prefetch -- chains, decoder parity tests, bench; kernarg placement A/B
mkdir -p gpurun_out
cd spittle_amd
for k in 1 2 3 4 5; do timeout -k 5 60 ./ubench_stamp chain $k 48 || exit 1; timeout -k 5 60 ./ubench chain $k 48 || exit 1; done
for v in 0 1; do HIP_FORCE_DEV_KERNARG=$v timeout -k 5 60 ./ubench chain 1 48 | sed "s/^/kernarg=$v /" || exit 1; done
cd ..
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "not free_running" > gpurun_out/t_r2b.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency > gpurun_out/bench_r2b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2b.log').read().strip().splitlines()[-1]);print('RTFx',d['value'],'dev',d['value_device_resident'],d['phases_ms'],d['rooflines']['decode_pass']['ms_per_pass'])"
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --no-probe --steps 5 | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('kernarg=1 RTFx',d['value'],d['phases_ms'])"
