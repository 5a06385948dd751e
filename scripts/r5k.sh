# round 5: B = 1 app-shape rocprofv3 summaries (chain, persistent) with an 8-row workspace
bash scripts/gpu_steps.sh \
 "r5k_b1|300|SPT_PERSISTENT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k_b1 -o prof -- python3 scripts/probe_b1.py" \
 "r5k_b1p|300|SPT_PERSISTENT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k_b1p -o prof -- python3 scripts/probe_b1.py" \
 "r5k_bench|400|python -u bench.py --no-parakeet --no-turbo --no-cpu-baseline"
