# encoder attention K-swizzle A/B (probe) + bf16 encoder parity
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 3 1 3; do
  SPT_ATTN_SWZ=$v timeout -k 10 120 python3 scripts/probe_kernels.py enc_attn > gpurun_out/probe_swz$v.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/probe_swz$v.log; exit 1; }
  echo "swz=$v $(tail -1 gpurun_out/probe_swz$v.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "encoder_bf16 or teacher_forced or batch_invariance" --timeout 120 --timeout-method thread > gpurun_out/g3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g3_tests.log; exit $rc
