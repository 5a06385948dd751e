set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1_tests.log 2>&1; rc=$?; tail -3 gpurun_out/t1_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/t1_bench.log 2>&1 && tail -1 gpurun_out/t1_bench.log &&
SPT_DECODE_GROUPS=2 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/t1_bench_g2.log 2>&1 && tail -1 gpurun_out/t1_bench_g2.log
