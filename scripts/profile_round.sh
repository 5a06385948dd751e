#!/bin/bash
# Round artefacts on the GPU box: full -m gpu suite, the default bench line (CPU baseline and app
# latency included), rocprofv3 kernel-trace stats of the same bench command, PMC traffic passes.
# usage: bash scripts/profile_round.sh TAG
TAG=${1:-r2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench_line.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
rm -f gpurun_out/${TAG}_prof/run_kernel_trace.csv
bash scripts/pmc.sh ${TAG} || exit 1
echo done
