#!/bin/bash
# GPU box: 128 x 128 GEMM LDS ring depth A/B (SPT_GEMM_NT_STAGES = 2 / 3 / 4) on the Parakeet bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for s in 2 4 3 4 2; do
  SPT_GEMM_NT_STAGES=$s timeout -k 10 300 python -u bench.py --parakeet-only --no-cpu-baseline --steps 5 --warmup 1 \
    > gpurun_out/r3e_st$s.json 2> gpurun_out/r3e_st$s.err || { echo "bench st=$s failed"; tail -5 gpurun_out/r3e_st$s.err; exit 1; }
  python3 - "$s" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r3e_st{sys.argv[1]}.json").read().strip().splitlines()[-1])
def walk(o, p=""):
    if isinstance(o, dict):
        for k, v in o.items(): walk(v, p + "." + k)
    elif isinstance(o, (int, float)) and any(t in p for t in ("ms", "rtfx", "value", "frac")):
        print(f"st={sys.argv[1]} {p} {o}")
walk(d)
PY
done
