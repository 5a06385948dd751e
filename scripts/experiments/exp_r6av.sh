#!/bin/bash
# r6av: Parakeet pending-slab LayerNorms with 1 / 2 waves per workgroup (SPT_LN_WPB) vs 4;
# bitwise test (tokens / top-1 of the fp16 C5 batch), then alternating Parakeet bench lines.
bash scripts/gpu_steps.sh \
  "r6av_tests|300|SPT_LN_WPB=1 python3 -u -m pytest tests/test_gpu_parakeet.py -m gpu -x -q -k 'bitwise or c5_streaming' --timeout 300 --timeout-method thread" \
  "r6av_w4a|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6av_w1a|300|SPT_LN_WPB=1 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6av_w2a|300|SPT_LN_WPB=2 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6av_w4b|300|python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6av_w1b|300|SPT_LN_WPB=1 python3 bench.py --parakeet-only --no-cpu-baseline" \
  "r6av_w2b|300|SPT_LN_WPB=2 python3 bench.py --parakeet-only --no-cpu-baseline"
