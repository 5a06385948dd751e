#!/bin/bash
# Round artefacts, part B (GPU box): rocprofv3 kernel-trace stats of the bench command, then the
# PMC traffic passes (scripts/pmc.sh).  usage: bash scripts/round_b.sh TAG
TAG=${1:-r4}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
rm -f gpurun_out/${TAG}_prof/run_kernel_trace.csv
bash scripts/pmc.sh ${TAG} || exit 1
echo done
