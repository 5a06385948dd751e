# round 5: encoder GEMM A/B (256- vs 240-row tile, and 4096^3 against the guide's 8-phase template),
# the default bench line, its rocprofv3 kernel stats, then the whole -m gpu suite
bash scripts/gpu_steps.sh \
 "r5e_ub|240|./spittle_amd/ubench gemm 4096 4096 4096 0 1 1 && for r in 256 240; do for a in '12000 3840 1280 0 1 1' '12000 5120 1280 1 1 1' '12000 1280 5120 3 1 1' '12000 1280 1280 3 1 1'; do SPT_G2_ROWS=\$r ./spittle_amd/ubench gemm \$a || exit 1; done; done" \
 "r5e_bench|400|python -u bench.py" \
 "r5e_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r5e_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe" \
 "r5e_tests|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
