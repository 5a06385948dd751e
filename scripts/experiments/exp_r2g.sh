#!/bin/bash
# r2: software-pipelined encoder attention (SPT_ENC_ATTN_PIPE=1 default) vs the r2 kernel
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ggml.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r2g.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2g.log; [ $rc -eq 0 ] || exit $rc
for P in 1 0; do
SPT_ENC_ATTN_PIPE=$P timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --steps 5 > gpurun_out/bench_r2g.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2g.log').read().strip().splitlines()[-1]);print('pipe=$P RTFx',d['value'],'enc',d['phases_ms']['encoder_ms'],d['rooflines']['encoder']['frac'],'attn',d['kernels']['enc_attn']['avg_us'],d['kernels']['enc_attn']['frac'])"
done
