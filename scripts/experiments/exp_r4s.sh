# r4s: (1) whisper_full's vocabulary statistics over 16 workgroups per row (dec_ts_stats) merged by
# finalize_ts -- the whisper_full / beam / parity tests; (2) the logits GEMV with 8 column tiles per
# workgroup (SPT_GV_LOGITS_CT=8: half the workgroups stage the final LayerNorm image, one wave per
# tile over all of K either way) -- bench lines A/B and the full-size bitwise tests under CT=8;
# (3) the beam candidates over 16 workgroups per row + a one-wave merge -- kernel stats of a beam call
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_full_large.py tests/test_gpu_ggml.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s/tests_full.log 2>&1 || { tail -30 gpurun_out/r4s/tests_full.log; exit 1; }
tail -1 gpurun_out/r4s/tests_full.log
for ct in 4 8; do
  SPT_GV_LOGITS_CT=$ct timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4s/bench_$ct.log 2>&1 || { tail -5 gpurun_out/r4s/bench_$ct.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4s/bench_$ct.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('CT=$ct', 'rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], 'logits_us', d['kernels']['dec_logits']['avg_us'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
done
SPT_GV_LOGITS_CT=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s/tests_ct8.log 2>&1 || { tail -30 gpurun_out/r4s/tests_ct8.log; exit 1; }
tail -1 gpurun_out/r4s/tests_ct8.log
MODE=beam timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s/prof_beam -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4s/prof_beam.log 2>&1 || { grep -v "^    @" gpurun_out/r4s/prof_beam.log | tail -20; exit 1; }
grep -E "^beam " gpurun_out/r4s/prof_beam.log
