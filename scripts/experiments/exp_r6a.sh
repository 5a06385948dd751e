#!/bin/bash
# r6a: C2 decode-pass traffic + a short bench (C2 line), then the run_decode SIGSEGV (VERDICT r5
# item 1): the library initialises HIP itself (no torch), first unprofiled, then under rocprofv3;
# a fault writes backtrace + maps to gpurun_out/segv_*.txt.
bash scripts/gpu_steps.sh \
  "r6a_c2pmc|500|bash scripts/c2_pmc.sh" \
  "r6a_bench|400|python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-turbo --no-parakeet" \
  "r6a_b1_plain|240|python3 scripts/probe_b1.py" \
  "r6a_b1_prof|300|B1_SEGV_OUT=gpurun_out/segv_b1_prof.txt rocprofv3 --kernel-trace --stats -d gpurun_out/r6a_prof -o prof -- python3 scripts/probe_b1.py"
