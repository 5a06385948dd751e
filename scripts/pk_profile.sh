#!/bin/bash
# GPU box: Parakeet-V3 bench line + rocprofv3 kernel stats of the same workload.
set -o pipefail
TAG=${1:-pk}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u bench.py --parakeet-only --steps 5 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 2500 gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 bench.py --parakeet-only --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
python3 - "$TAG" <<'PY'
import csv, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/{tag}_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
with open(f"gpurun_out/{tag}_kernel_top.txt", "w") as f:
    for r in rows[:25]:
        line = f'{float(r["TotalDurationNs"])/tot*100:6.2f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f}us  {r["Name"][:150]}'
        print(line); f.write(line + "\n")
PY
find gpurun_out/${TAG}_prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
