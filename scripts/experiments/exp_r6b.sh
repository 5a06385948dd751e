#!/bin/bash
# r6b: (1) the rocprofv3 fault in hipGraphLaunch (r6a: inside librocprofiler-sdk's packet intercept,
# called from libhsa-runtime64, under the system HIP 7.2 runtime): eager passes (no graph launch) and
# the 7.2 runtime's graph batching turned off, both under rocprofv3 without torch; (2) persistent-pass
# stage stamps at B = 1 and B = 8.
bash scripts/gpu_steps.sh \
  "r6b_pd_b1|240|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1.bin python3 scripts/probe_b1.py" \
  "r6b_pd_b8|240|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b8.bin B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6b_pd_b1_nostamp|240|SPT_PERSISTENT=1 python3 scripts/probe_b1.py" \
  "r6b_prof_eager|300|SPT_NO_GRAPH=1 B1_SEGV_OUT=gpurun_out/segv_r6b_eager.txt rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_eager -o prof -- python3 scripts/probe_b1.py" \
  "r6b_prof_gb1|300|DEBUG_HIP_GRAPH_BATCH_SIZE=1 B1_SEGV_OUT=gpurun_out/segv_r6b_gb1.txt rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_gb1 -o prof -- python3 scripts/probe_b1.py"
