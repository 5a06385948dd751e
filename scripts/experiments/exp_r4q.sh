# r4q: beam steps upload their row state / step / sources in one copy and read their candidates back
# in one copy (consecutive workspace carvings); the beam tests and a bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_full_large.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1 || { tail -30 gpurun_out/r4q/tests.log; exit 1; }
tail -1 gpurun_out/r4q/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4q/bench.log 2>&1 || { tail -5 gpurun_out/r4q/bench.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4q/bench.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms'], a[k]['host_ms']) for k in a})"
