# round 5: decoder LayerNorm-prologue GEMVs with two column tiles per workgroup below N = 4096
# (SPT_GV_CT2_MIN = 3840: q/k/v too; 1280: q/k/v and cross-Q), alternating A/B bench runs
bash scripts/gpu_steps.sh \
 "r5ak_d1|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ak_q1|300|SPT_GV_CT2_MIN=3840 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ak_a1|300|SPT_GV_CT2_MIN=1280 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ak_d2|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ak_q2|300|SPT_GV_CT2_MIN=3840 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5ak_a2|300|SPT_GV_CT2_MIN=1280 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
