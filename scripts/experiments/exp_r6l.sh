#!/bin/bash
# r6l: r6k's measurements again with the rocprofv3 databases summarised on the box and removed (r6k's
# two whole-bench traces took gpurun_out past the 64 MiB copy-back limit): the default bench line, the
# encoder probes against rocprofv3 over the same launches (one window group), the default bench's
# kernel stats, the PMC traffic.
B="python3 bench.py --steps 5 --warmup 2"
Q="--no-c2 --no-parakeet --no-turbo --no-app-latency --no-cpu-baseline"
bash scripts/gpu_steps.sh \
  "r6l_bench|600|$B" \
  "r6l_probe_prof|400|SPT_ENC_GROUPS=1 DEBUG_HIP_GRAPH_BATCH_SIZE=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r6l_probe_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q" \
  "r6l_probe_cmp|120|python3 scripts/probe_vs_rocprof.py gpurun_out/r6l_probe_prof/prof_results.db gpurun_out/r6l_probe_prof.log 50 && python3 scripts/rocpd_top.py gpurun_out/r6l_probe_prof/prof_results.db 40 && rm -rf gpurun_out/r6l_probe_prof" \
  "r6l_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r6l_prof -o prof -- python3 bench.py --steps 3 --warmup 1 $Q --no-probe" \
  "r6l_prof_top|120|python3 scripts/rocpd_top.py gpurun_out/r6l_prof/prof_results.db 60 4 && rm -rf gpurun_out/r6l_prof" \
  "r6l_pmc|700|bash scripts/pmc.sh r6l"
