#!/bin/bash
# r6ak: per-kernel profile of the Parakeet C5 streaming pass (bench.py --parakeet-only, summarised on the box).
bash scripts/gpu_steps.sh \
  "r6ak_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r6ak_prof -o prof -- python3 bench.py --parakeet-only --no-cpu-baseline --steps 5 --warmup 2" \
  "r6ak_top|120|python3 scripts/rocpd_top.py gpurun_out/r6ak_prof/prof_results.db 40 && rm -rf gpurun_out/r6ak_prof"
