#!/bin/bash
# r2: lazy softmax rescale in the encoder attention; C2 (small f32 B=1) and C1-dims (tiny.en) lines
mkdir -p gpurun_out
cd spittle_amd && timeout -k 5 120 ./ubench gemm 12000 3840 1280 0 1 >/dev/null; cd ..
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_ggml.py -x -q --timeout 300 --timeout-method thread -k "not free_running" > gpurun_out/t_r2f.log 2>&1; rc=$?; tail -3 gpurun_out/t_r2f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-app-latency --steps 5 > gpurun_out/bench_r2f.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_r2f.log').read().strip().splitlines()[-1]);print('RTFx',d['value'],d['phases_ms'],d['rooflines']['encoder']['frac'],d['kernels']['enc_attn'])"
timeout -k 10 300 python -u bench.py --model synthetic:small --dtype f32 --batch 1 --no-app-latency > gpurun_out/bench_c2_small.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c2_small.log > gpurun_out/bench_line_c2_small_f32.json
timeout -k 10 300 python -u bench.py --model synthetic:tiny.en --dtype f32 --batch 1 --no-app-latency --no-probe > gpurun_out/bench_c1_tiny.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c1_tiny.log > gpurun_out/bench_line_tiny_en_f32.json
echo done
