# r4k (and r4l: the vocabulary kernels on register-resident logits, the A_ATTN merge in batches of four): beam step -- one query per workgroup for shared one-token steps (cross-attention) and the
# one-pass beam candidate kernel, one self-K/V gather per step (alternating sides); tests, the beam
# case, the bench line, kernel stats of the beam call
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
T="tests/test_gpu_fullsize.py tests/test_gpu_full.py tests/test_gpu_full_large.py tests/test_gpu_parity.py tests/test_gpu_multi.py"
timeout -k 10 600 python -u -m pytest $T -q --timeout 300 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4k/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 120 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4k/beam.log 2>&1 || { tail -20 gpurun_out/r4k/beam.log; exit 1; }
grep -h "^env" gpurun_out/r4k/beam.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4k/bench.log 2>&1 || { tail -5 gpurun_out/r4k/bench.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4k/bench.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], 'xattn', d['roofline']['avg_us'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
MODE=beam timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k/prof_beam -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4k/prof_beam.log 2>&1 || { grep -v "^    @" gpurun_out/r4k/prof_beam.log | tail -20; exit 1; }
grep -E "^beam " gpurun_out/r4k/prof_beam.log
