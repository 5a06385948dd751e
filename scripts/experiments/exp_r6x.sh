#!/bin/bash
# r6x: f32 64-row tiles now the default below a full round of 128 x 128 tiles: encoder output bitwise
# against SPT_GEMM_F32_SMALL=0 (tiny and small f32), the f32 / full-pipeline suites, and the C2 bench
# entry (bench.py runs it by default; this line skips the other configs).
bash scripts/gpu_steps.sh \
  "r6x_dump_small_0|200|SPT_GEMM_F32_SMALL=0 python3 scripts/enc_dump.py synthetic:small f32 gpurun_out/r6x_small_0.npz" \
  "r6x_dump_small_1|200|python3 scripts/enc_dump.py synthetic:small f32 gpurun_out/r6x_small_1.npz" \
  "r6x_dump_tiny_0|200|SPT_GEMM_F32_SMALL=0 python3 scripts/enc_dump.py synthetic:tiny.en f32 gpurun_out/r6x_tiny_0.npz" \
  "r6x_dump_tiny_1|200|python3 scripts/enc_dump.py synthetic:tiny.en f32 gpurun_out/r6x_tiny_1.npz" \
  "r6x_cmp|60|python3 -c \"import numpy as np
for m in ('small', 'tiny'):
    a, b = np.load('gpurun_out/r6x_%s_0.npz' % m)['enc'], np.load('gpurun_out/r6x_%s_1.npz' % m)['enc']
    print(m, 'bitwise', bool(np.array_equal(a, b)), 'max abs diff', float(np.abs(a - b).max()))\"" \
  "r6x_tests|700|python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_ggml.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r6x_bench_c2|400|python3 bench.py --steps 5 --warmup 2 --no-parakeet --no-turbo --no-app-latency"
