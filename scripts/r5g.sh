# round 5: GEMM with the DMA issued before each phase's fragment reads (ubench, bitwise vs 128-tile),
# stagger on/off; rocprofv3 of the bench (Q-in-LDS attention, 256-row tiles)
bash scripts/gpu_steps.sh \
 "r5g_ub|240|for a in '4096 4096 4096 0 1 1' '12000 3840 1280 0 1 1' '12000 5120 1280 1 1 1' '12000 1280 5120 3 1 1'; do ./spittle_amd/ubench gemm \$a || exit 1; SPT_G2_STAGGER=0 ./spittle_amd/ubench gemm \$a || exit 1; done" \
 "r5g_prof|400|rocprofv3 --kernel-trace --stats -d gpurun_out/r5g_prof -o prof -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet --no-turbo"
