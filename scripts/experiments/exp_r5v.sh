# round 5: encoder window groups A/B (alternating G=1 / G=2, C3 bench), and the encoder kernels'
# effective clock under profiling (GRBM_GUI_ACTIVE)
bash scripts/gpu_steps.sh \
 "r5v_g1a|300|SPT_ENC_GROUPS=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5v_g2a|300|SPT_ENC_GROUPS=2 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5v_g1b|300|SPT_ENC_GROUPS=1 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5v_g2b|300|SPT_ENC_GROUPS=2 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5v_clk|200|bash scripts/pmc_clock.sh"
