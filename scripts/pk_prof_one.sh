#!/bin/bash
# GPU box: rocprofv3 kernel stats of one Parakeet workload (PK_BENCH_ONLY=offline|stream).
set -o pipefail
W=${1:-offline}; TAG=${2:-pkw}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PK_BENCH_ONLY=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
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
    for r in rows[:22]:
        line = f'{float(r["TotalDurationNs"])/tot*100:6.2f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f}us  {r["Name"][:110]}'
        print(line); f.write(line + "\n")
PY
find gpurun_out/${TAG}_prof -name "*.csv" ! -name "*kernel_stats.csv" -delete
