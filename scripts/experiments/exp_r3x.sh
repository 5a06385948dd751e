# r3 s2: small-M GEMM tiles (64 x 128, then 64 x 64; Parakeet C5 incl. residual products; Whisper single-window
# encoder through the automatic tile choice): ubench shapes, the whole GPU suite, the Parakeet lines
# with and without the tile (SPT_GEMM_T64=0), and the default bench line (app-call latency included)
export TMPDIR=/tmp
mkdir -p gpurun_out
U=spittle_amd/ubench
for cfg in "1500 1280 1280 3 1" "1500 1280 5120 3 1" "1500 3840 1280 0 1" "1500 5120 1280 1 1" "3000 1280 384 2 1" "1500 1280 3840 2 1" "12000 1280 1280 3 1"; do
  timeout -k 5 60 $U gemm $cfg || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { tail -20 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
for t in 1 0; do
  SPT_GEMM_T64=$t timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3x_pk$t.log 2>&1 || { tail -5 gpurun_out/r3x_pk$t.log; exit 1; }
done
timeout -k 10 500 python3 bench.py --no-cpu-baseline > gpurun_out/r3x_bench.log 2>&1 || { tail -5 gpurun_out/r3x_bench.log; exit 1; }
echo bench done
