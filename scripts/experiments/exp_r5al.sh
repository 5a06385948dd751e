# round 5: fc1 with one column tile per workgroup (SPT_GV_CT2_MIN = 8192) against the default two, alternating
bash scripts/gpu_steps.sh \
 "r5al_d1|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5al_f1|300|SPT_GV_CT2_MIN=8192 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5al_d2|300|python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe" \
 "r5al_f2|300|SPT_GV_CT2_MIN=8192 python -u bench.py --steps 8 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-probe"
