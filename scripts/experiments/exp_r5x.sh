# round 5: decoder cross-attention key split over workgroups (SPT_XATTN_SPLIT, merged by the cross-out
# GEMV prologue) re-measured at C3 on the r5 tree
bash scripts/gpu_steps.sh \
 "r5x_s1|300|python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5x_s2|300|SPT_XATTN_SPLIT=2 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5x_s3|300|SPT_XATTN_SPLIT=3 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5x_s4|300|SPT_XATTN_SPLIT=4 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
