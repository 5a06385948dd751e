# r3 s2: TDT decode with 16-row passes for batches over 8 (one pass per workgroup) vs 8-row passes
# (SPT_PK_DEC_DR8=1); the whole GPU suite first (also covers the removal of the fused-QKV variant)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ac_tests.log 2>&1 || { tail -20 gpurun_out/r3ac_tests.log; exit 1; }
tail -1 gpurun_out/r3ac_tests.log
for v in 0 1; do
  if [ $v = 1 ]; then export SPT_PK_DEC_DR8=1; fi
  PK_BENCH_ONLY=stream64 timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3ac_pk$v.log 2>&1 || { tail -5 gpurun_out/r3ac_pk$v.log; exit 1; }
done
echo bench done
