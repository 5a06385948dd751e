# round 5: the -m gpu suite with the ping-pong GEMM default, then B = 1 rocprofv3 diagnostics (the
# profiled B = 1 fast path crashed in the HIP runtime in r5i / r5k; without the profiler it runs)
bash scripts/gpu_steps.sh \
 "r5n_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r5n_b1vw0|200|SPT_XATTN_VW=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r5n_b1vw0 -o prof -- python3 scripts/probe_b1.py" \
 "r5n_b1ng|300|SPT_NO_GRAPH=1 rocprofv3 --kernel-trace --stats -d gpurun_out/r5n_b1ng -o prof -- python3 scripts/probe_b1.py"
