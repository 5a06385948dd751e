# r3 s2: LayerNorm loads issued up front (x, gamma, beta) and the TDT decode stages' row groups
# spread over grid.y: parity tests, Parakeet bench + stream64 kernel stats, Whisper encoder time
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1 || { tail -20 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3q_pk.log 2>&1 || { tail -5 gpurun_out/r3q_pk.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3q_pk.log').read().strip().splitlines()[-1])['parakeet']; print({k: (v.get('rtfx'), v.get('phases_ms')) for k, v in d.items() if isinstance(v, dict) and 'phases_ms' in v})"
PK_BENCH_ONLY=stream64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3q_prof -o run -- python3 bench.py --parakeet-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3q_prof.log 2>&1 || { tail -5 gpurun_out/r3q_prof.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3q_prof/run_kernel_stats.csv 12
rm -f gpurun_out/r3q_prof/run_kernel_trace.csv
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-app-latency --no-probe > gpurun_out/r3q_bench.log 2>&1 || { tail -5 gpurun_out/r3q_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3q_bench.log').read().strip().splitlines()[-1]); print(d['value'], d.get('phases_ms'), d.get('rooflines', {}).get('encoder'))"
