# round 5 final tree: rocprofv3 kernel stats of the bench (C3 + turbo + Parakeet lines), a B = 1
# app-call profile, then the whole -m gpu suite
bash scripts/gpu_steps.sh \
 "r5i_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r5i_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe" \
 "r5i_b1|300|SPT_PERSISTENT=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5i_b1 -o prof -- python3 scripts/probe_b1.py" \
 "r5i_b1p|300|SPT_PERSISTENT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r5i_b1p -o prof -- python3 scripts/probe_b1.py" \
 "r5i_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
