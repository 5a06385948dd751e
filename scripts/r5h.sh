# round 5: ring GEMM with three K-steps in flight (ubench at the C5 shapes), its C5 bench line, and
# the default bench line of the tree
bash scripts/gpu_steps.sh \
 "r5h_ub|200|for a in '832 4096 1024 5 2 1' '832 3072 1024 0 2 1' '832 2048 1024 0 2 1' '832 1024 4096 8 2 4' '832 1024 1024 8 2 4'; do SPT_RING_D=3 ./spittle_amd/ubench gemm \$a || exit 1; done" \
 "r5h_pk3|300|SPT_GEMM_RING=1 SPT_RING_D=3 python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5h_bench|400|python -u bench.py"
