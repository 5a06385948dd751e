# r3 s2: Parakeet encoder stage profile (ABI 10) -- parity + C smoke tests, then the Parakeet bench
# lines with their per-stage rooflines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py tests/test_capi_c.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1 || { tail -20 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
timeout -k 10 400 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3s_pk.log 2>&1 || { tail -5 gpurun_out/r3s_pk.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3s_pk.log').read().strip().splitlines()[-1])['parakeet']
for k in ('streaming_1s_b64', 'offline_30s_b8'):
    v = d[k]; print(k, v['rtfx'], v['phases_ms']['encoder_ms'], v['encoder_roofline']['frac'])
    for s, r in v['kernels'].items(): print('   ', s, r)
"
