# r4p: beam candidates kept in LDS until the rounds end, branch-free mask bits, the cross-attention
# strategy switch read per capture (+ the cross-strategy bitwise tests); the beam tests and
# kernel stats of the beam call
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_full_large.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4p/tests.log 2>&1 || { tail -30 gpurun_out/r4p/tests.log; exit 1; }
tail -1 gpurun_out/r4p/tests.log
MODE=beam timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p/prof_beam -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4p/prof_beam.log 2>&1 || { grep -v "^    @" gpurun_out/r4p/prof_beam.log | tail -20; exit 1; }
grep -E "^beam " gpurun_out/r4p/prof_beam.log
