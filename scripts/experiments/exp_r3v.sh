# r3 s2 (second run: the 64 x 128 tile also for the residual products, >= 8 K-steps per split): 64 x 128 GEMM tile (variant 4) at the Parakeet C5 shapes: ubench timing + bitwise check
# against the 128 x 128 tile, Parakeet parity, then the C5 / offline bench with it (default) and
# without it (SPT_GEMM_T64=0)
export TMPDIR=/tmp
mkdir -p gpurun_out
U=spittle_amd/ubench
for cfg in "832 4096 1024 5 2" "832 1024 4096 8 2 4" "832 1024 1024 8 2 2" "832 4096 1024 0 1"; do
  timeout -k 5 60 $U gemm $cfg || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1 || { tail -20 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
for t in 1 0 1 0; do
  SPT_GEMM_T64=$t timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3v_pk$t.log 2>&1 || { tail -5 gpurun_out/r3v_pk$t.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3v_pk$t.log').read().strip().splitlines()[-1])['parakeet']
for k in ('streaming_1s_b64', 'offline_30s_b8'):
    v = d[k]; print('T64=$t', k, v['rtfx'], v['phases_ms']['encoder_ms'], v['encoder_roofline']['frac'], {s: (r['ms'] if isinstance(r, dict) else r) for s, r in v['kernels'].items()})
"
done
