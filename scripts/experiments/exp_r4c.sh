# r4c: cross-attention grid and register ring, all bitwise the same result by construction:
#  SPT_XATTN_VW=1 (default): 8 single-wave workgroups per (window run, head) when the 8-wave grid is
#    small (B = 1, shared windows), merged by the cross-out GEMV's A_ATTN prologue; 0: never; 2: always
#  SPT_XATTN_PF=2..4: key blocks in each wave's register ring (PF - 1 loading ahead)
# the cross-strategy bitwise tests (default and VW=2 PF=4), then the latency lines per setting
export TMPDIR=/tmp
mkdir -p gpurun_out
T="tests/test_gpu_fullsize.py tests/test_gpu_full.py tests/test_gpu_full_large.py tests/test_gpu_multi.py tests/test_gpu_parity.py"
timeout -k 10 500 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
SPT_XATTN_VW=2 SPT_XATTN_PF=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c_tests_vw2pf4.log 2>&1 || { tail -30 gpurun_out/r4c_tests_vw2pf4.log; exit 1; }
tail -1 gpurun_out/r4c_tests_vw2pf4.log
for cfg in 1:2 0:2 2:2 1:4 2:4 2:3; do
  v=${cfg%%:*}; pf=${cfg##*:}
  SPT_XATTN_VW=$v SPT_XATTN_PF=$pf timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4c_bench_${v}_$pf.log 2>&1 || { tail -5 gpurun_out/r4c_bench_${v}_$pf.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4c_bench_${v}_$pf.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('VW=$v PF=$pf', 'rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
done
