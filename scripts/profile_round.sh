#!/bin/bash
# Round artefacts on the GPU box: bench line (with the CPU baseline), rocprofv3 kernel-trace
# stats of the same bench command, PMC HBM traffic passes.  usage: bash scripts/profile_round.sh TAG
TAG=${1:-r1}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench_line.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
bash scripts/pmc.sh ${TAG} || exit 1
echo done
