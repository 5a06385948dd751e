#!/bin/bash
# GPU-box check: parity tests, a bench line, and a rocprofv3 kernel-stats profile.
# usage: bash scripts/gpu_check.sh TAG [bench args...]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
