SKIP_PROF=1 bash scripts/gpu_check.sh r4b && bash scripts/experiments/exp_r4a.sh
