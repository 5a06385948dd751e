# round 5: B = 1 rocprofv3 summaries (torch-initialised process), then SQ issue / wait counters of
# the encoder attention and fc1 GEMM
bash scripts/gpu_steps.sh \
 "r5p_b1|300|SPT_PERSISTENT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p_b1 -o prof -- python3 scripts/probe_b1.py" \
 "r5p_b1p|300|SPT_PERSISTENT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r5p_b1p -o prof -- python3 scripts/probe_b1.py" \
 "r5p_sq|400|bash scripts/pmc_sq.sh"
