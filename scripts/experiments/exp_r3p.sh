# r3 s2: Parakeet conv module with unconditional (clamped) loads: parity tests, then the Parakeet bench
# lines (streaming 64 x 1 s, offline 8 x 30 s) and a kernel-stats profile of the offline pass
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || { tail -20 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3p_bench.log 2>&1 || { tail -5 gpurun_out/r3p_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3p_bench.log').read().strip().splitlines()[-1])['parakeet']; print({k: (v.get('rtfx'), v.get('phases_ms', {}).get('encoder_ms'), v.get('encoder_roofline', {}).get('frac')) for k, v in d.items() if isinstance(v, dict) and 'phases_ms' in v})"
PK_BENCH_ONLY=offline timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3p_prof -o run -- python3 bench.py --parakeet-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3p_prof.log 2>&1 || { tail -5 gpurun_out/r3p_prof.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3p_prof/run_kernel_stats.csv 14
rm -f gpurun_out/r3p_prof/run_kernel_trace.csv
