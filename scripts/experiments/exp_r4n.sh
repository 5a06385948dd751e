# r4n: key blocks in flight per cross-attention wave (SPT_XATTN_PF = 2 / 3 / 4: the single-wave
# kernels of B = 1 and of a beam's per-query steps; no result changes), bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
for pf in 2 3 4; do
  SPT_XATTN_PF=$pf timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4n/bench_$pf.log 2>&1 || { tail -5 gpurun_out/r4n/bench_$pf.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4n/bench_$pf.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('PF=$pf', 'rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], 'xattn', d['roofline']['avg_us'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
done
