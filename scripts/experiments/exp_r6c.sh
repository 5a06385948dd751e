#!/bin/bash
# r6c: the encoder LayerNorm fold (A/B against SPT_LN_FOLD=0), persistent-pass stage stamps, then
# the whole -m gpu suite.
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-parakeet --no-turbo --no-c2"
bash scripts/gpu_steps.sh \
  "r6c_bench_fold|300|$B" \
  "r6c_bench_nofold|300|SPT_LN_FOLD=0 $B" \
  "r6c_pd_b1|240|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b1.bin python3 scripts/probe_b1.py" \
  "r6c_pd_b8|240|SPT_PERSISTENT=1 SPT_PD_STAMP=gpurun_out/pd_stamps_b8.bin B1_BATCH=8 python3 scripts/probe_b1.py" \
  "r6c_tests|900|python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
