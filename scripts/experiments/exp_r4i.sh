# r4i: the straight-line attention schedule with its arithmetic pinned (contraction off, explicit
# fmaf): bitwise / parity tests, the beam case, the bench line, kernel stats of beam-5 and B = 1 calls
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
T="tests/test_gpu_fullsize.py tests/test_gpu_full.py tests/test_gpu_full_large.py tests/test_gpu_parity.py tests/test_gpu_multi.py"
timeout -k 10 600 python -u -m pytest $T -q --timeout 300 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4i_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4i_beam.log 2>&1 || { tail -20 gpurun_out/r4i_beam.log; exit 1; }
grep -h "^env" gpurun_out/r4i_beam.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4i_bench.log 2>&1 || { tail -5 gpurun_out/r4i_bench.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4i_bench.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], 'xattn', d['roofline']['avg_us'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
for m in beam b1; do
  MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d/$m -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4d/$m.log 2>&1 || { tail -20 gpurun_out/r4d/$m.log; exit 1; }
  grep -E "^(beam|b1) " gpurun_out/r4d/$m.log
done
