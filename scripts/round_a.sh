#!/bin/bash
# Round artefacts, part A (GPU box): the full -m gpu suite and the default bench line.
# usage: bash scripts/round_a.sh TAG   (part B: scripts/round_b.sh TAG -- kernel stats + PMC passes)
TAG=${1:-r4}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench_line.json
echo done
