#!/bin/bash
# r6y: per-kernel profile of the C2 call (Whisper-small f32, B = 1): scripts/c2_probe.py under rocprofv3
# (database summarised on the box).
bash scripts/gpu_steps.sh \
  "r6y_prof|300|rocprofv3 --kernel-trace --stats -d gpurun_out/r6y_prof -o prof -- python3 scripts/c2_probe.py" \
  "r6y_top|120|python3 scripts/rocpd_top.py gpurun_out/r6y_prof/prof_results.db 45 && rm -rf gpurun_out/r6y_prof"
