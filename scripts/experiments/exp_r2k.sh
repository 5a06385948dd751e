# r2 session 3: fused QKV + self-attention, LayerNorm row staged through LDS and an 8-unit weight ring (bitwise test, bench A/B)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_qkv.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fused_test.log 2>&1
rc=$?; tail -3 gpurun_out/fused_test.log; [ $rc -eq 0 ] || exit $rc
run() {
  env "$@" timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/bench_k.log 2>&1 || { echo "bench failed: $*"; tail -5 gpurun_out/bench_k.log; exit 1; }
  echo "$* $(tail -1 gpurun_out/bench_k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phases_ms"]["decode_ms"], d["rooflines"]["decode_pass"]["ms_per_pass"])')"
}
run SPT_FUSED_QKV=0
run SPT_FUSED_QKV=1 SPT_FUSED_QKV_ROT=0
run SPT_FUSED_QKV=1 SPT_FUSED_QKV_ROT=1
