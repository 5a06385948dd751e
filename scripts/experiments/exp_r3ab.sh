# r3 s2: Parakeet block-boundary LayerNorm pair fused (ln_pend2_kernel); earlier runs of this script: relative attention variants (wave-local sync + loads before products kept; one-tile-ahead prefetch measured slower, 0.96 -> 1.27 ms offline, dropped)
# tile's K / position rows issued before its products (sched_barrier): parity, then the Parakeet lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ab_tests.log 2>&1 || { tail -20 gpurun_out/r3ab_tests.log; exit 1; }
tail -1 gpurun_out/r3ab_tests.log
timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3ab_pk.log 2>&1 || { tail -5 gpurun_out/r3ab_pk.log; exit 1; }
echo bench done
