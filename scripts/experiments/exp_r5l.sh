# round 5: ping-pong GEMM phases (SPT_G2_PP=1) against the staggered default, standalone, bitwise vs 128-tile
bash scripts/gpu_steps.sh \
 "r5l_ub|300|for a in '4096 4096 4096 0 1 1' '12000 3840 1280 0 1 1' '12000 5120 1280 1 1 1' '12000 1280 5120 3 1 1' '12000 1280 1280 3 1 1'; do ./spittle_amd/ubench gemm \$a || exit 1; SPT_G2_PP=1 ./spittle_amd/ubench gemm \$a || exit 1; done" \
 "r5l_bpp|300|SPT_G2_PP=1 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo"
