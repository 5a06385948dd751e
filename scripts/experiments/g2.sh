# session 2: resampler GPU parity, then SQ counters over the encoder kernels
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resampler.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/rs_tests.log 2>&1
rc=$?; tail -12 gpurun_out/rs_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sq.sh
