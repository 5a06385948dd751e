bash scripts/gpu_steps.sh \
 "r5d_ub|180|for a in '832 4096 1024 5 2 1' '832 3072 1024 0 2 1' '832 2048 1024 0 2 1' '832 1024 4096 8 2 4' '832 1024 1024 8 2 4' '832 1024 1024 8 2 2' '1500 1280 1280 3 1 1' '12000 3840 1280 0 1 1'; do ./spittle_amd/ubench gemm \$a || exit 1; done" \
 "r5d_pk|400|python -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -v --timeout 200 --timeout-method thread" \
 "r5d_bpk1|300|python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5d_bpk0|300|SPT_GEMM_RING=0 python -u bench.py --parakeet-only --no-cpu-baseline" \
 "r5d_vn|200|rocprofv3 --kernel-trace --stats -d gpurun_out/vn -o vn -- python3 scripts/vendor_gemm_names.py"
