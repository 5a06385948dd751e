bash scripts/gpu_steps.sh \
 "r5m_b1|200|SPT_TRACE_COPIES=1 SPT_PERSISTENT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m_b1 -o prof -- python3 scripts/probe_b1.py"
