# round 5: logits GEMV with every wave's K slice in flight (SPT_GV_LOGITS_CT=42: 8 waves, 4 column tiles,
# K split over 2 waves, 5 super-steps each, exact) against the default (4, 4, 4)
bash scripts/gpu_steps.sh \
 "r5z_d|300|python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo" \
 "r5z_42|300|SPT_GV_LOGITS_CT=42 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo" \
 "r5z_d2|300|python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo" \
 "r5z_42b|300|SPT_GV_LOGITS_CT=42 python -u bench.py --steps 6 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo"
