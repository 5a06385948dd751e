#!/bin/bash
# r6as: final tree after the Parakeet host-copy changes: whole -m gpu suite, smoke, two default bench lines, kernel stats
Q="--no-c2 --no-parakeet --no-turbo --no-app-latency --no-cpu-baseline --no-probe"
bash scripts/gpu_steps.sh \
  "r6as_tests|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6as_smoke|300|python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r6as_bench|600|python3 bench.py" \
  "r6as_bench2|600|python3 bench.py --steps 10 --warmup 3" \
  "r6as_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r6as_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q" \
  "r6as_prof_top|120|python3 scripts/rocpd_top.py gpurun_out/r6as_prof/prof_results.db 60 4 && rm -rf gpurun_out/r6as_prof"
