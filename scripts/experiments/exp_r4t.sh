# r4t: the attention waves' K/V offsets in 32-bit unsigned arithmetic (pure indexing: the same keys,
# the same bits): the decoder tests and a bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
T="tests/test_gpu_fullsize.py tests/test_gpu_full.py tests/test_gpu_full_large.py tests/test_gpu_parity.py tests/test_gpu_multi.py"
timeout -k 10 700 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t/tests.log 2>&1 || { tail -30 gpurun_out/r4t/tests.log; exit 1; }
tail -1 gpurun_out/r4t/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4t/bench.log 2>&1 || { tail -5 gpurun_out/r4t/bench.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4t/bench.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], 'xattn', d['roofline']['avg_us'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
