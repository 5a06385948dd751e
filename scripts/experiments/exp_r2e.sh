#!/bin/bash
# r2: blocked cross K/V layout in the engine -- decoder parity + bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_full.py tests/test_gpu_ggml.py -x -q --timeout 300 --timeout-method thread -k "not free_running" > gpurun_out/t_r2e.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --steps 5 > gpurun_out/bench_r2e.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2e.log').read().strip().splitlines()[-1]);print('RTFx',d['value'],d['phases_ms'],d['rooflines']['decode_pass']['ms_per_pass'], d['roofline']['avg_us'])"
