#!/bin/bash
# r6k: the round-6 tree after the deletions: the whole -m gpu suite, the default bench line, the
# encoder probes against rocprofv3 over the same launches (one window group), the default bench's
# kernel stats, and the PMC traffic of the hot-path kernels.
B="python3 bench.py --steps 5 --warmup 2"
Q="--no-c2 --no-parakeet --no-turbo --no-app-latency --no-cpu-baseline"
bash scripts/gpu_steps.sh \
  "r6k_tests|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6k_bench|600|$B" \
  "r6k_probe_prof|400|SPT_ENC_GROUPS=1 DEBUG_HIP_GRAPH_BATCH_SIZE=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_probe_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q" \
  "r6k_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q --no-probe" \
  "r6k_pmc|700|bash scripts/pmc.sh r6k"
