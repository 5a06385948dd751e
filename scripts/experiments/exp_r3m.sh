# r3 s2: 256x256 GEMM residual / positional epilogue with the f32 operand loaded before the stores
# (ubench, random bf16; 128-tile bitwise reference), then the encoder tests and a C3 bench
export TMPDIR=/tmp
for s in "12288 4096 1280 0" "12288 4096 1280 3" "12000 1280 1280 3" "12000 1280 5120 3" "12000 3840 1280 0" "12000 5120 1280 1"; do
  timeout -k 10 120 ./spittle_amd/ubench gemm $s 1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { tail -20 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-parakeet > gpurun_out/r3m_bench.log 2>&1 || { tail -5 gpurun_out/r3m_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3m_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['phases_ms'], d['rooflines']['encoder'])"
