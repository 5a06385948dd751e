# round 5: software-pipelined encoder attention (attn_bf16_sp_kernel: the next tile's QK^T beside
# this tile's softmax in one wave; SPT_ATTN_SP=1: 32 queries per wave, two waves per SIMD; =2: 64
# queries, one wave per SIMD): oracle parity, repeatability, probes against the default
bash scripts/gpu_steps.sh \
 "r5ae_p1|300|SPT_ATTN_SP=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'encoder_bf16 or transcribe_bf16'" \
 "r5ae_p2|300|SPT_ATTN_SP=2 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k 'encoder_bf16 or transcribe_bf16'" \
 "r5ae_r1|400|SPT_ATTN_SP=1 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k 'repeatable'" \
 "r5ae_a0|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5ae_a1|200|SPT_ATTN_SP=1 python3 scripts/probe_kernels.py enc_attn" \
 "r5ae_a2|200|SPT_ATTN_SP=2 python3 scripts/probe_kernels.py enc_attn" \
 "r5ae_a0b|200|python3 scripts/probe_kernels.py enc_attn" \
 "r5ae_a1b|200|SPT_ATTN_SP=1 python3 scripts/probe_kernels.py enc_attn"
