# round 5: B = 1 rocprofv3 diagnostics (app's whisper_full call on 10 s; the fast path eager), then the final bench line
bash scripts/gpu_steps.sh \
 "r5o_bench|400|python -u bench.py" \
 "r5o_b1full|300|B1_FULL=1 B1_SAMPLES=160000 SPT_PERSISTENT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5o_b1full -o prof -- python3 scripts/probe_b1.py" \
 "r5o_b1ng|300|SPT_NO_GRAPH=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r5o_b1ng -o prof -- python3 scripts/probe_b1.py"
