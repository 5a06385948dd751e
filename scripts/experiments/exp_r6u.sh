#!/bin/bash
# r6u: the round-6 tree after the self-attention prefetch: whole -m gpu suite, default bench line,
# kernel stats of the default bench (database summarised on the box), smoke.
Q="--no-c2 --no-parakeet --no-turbo --no-app-latency --no-cpu-baseline --no-probe"
bash scripts/gpu_steps.sh \
  "r6u_tests|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6u_smoke|300|python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "r6u_bench|600|python3 bench.py --steps 10 --warmup 3" \
  "r6u_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r6u_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q" \
  "r6u_prof_top|120|python3 scripts/rocpd_top.py gpurun_out/r6u_prof/prof_results.db 60 4 && rm -rf gpurun_out/r6u_prof"
