#!/bin/bash
# GPU-box check: parity tests, a bench line, and a rocprofv3 kernel-stats profile.
# usage: bash scripts/gpu_check.sh TAG [bench args...]   (SKIP_TESTS=1 to skip pytest)
TAG=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -5 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-turbo "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
fi
echo done
