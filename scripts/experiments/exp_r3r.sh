# r3 s2: TDT decode stages with the next row group's rows prefetched under the current group's
# products (weights waited before the loop), utterances per workgroup swept; LayerNorm in situ
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parakeet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1 || { tail -20 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
for rows in 16,16,32 8,8,8 32,32,64 16,16,16; do
  SPT_PK_DEC_ROWS=$rows PK_BENCH_ONLY=stream64 timeout -k 10 300 python3 bench.py --parakeet-only --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3r_pk_$rows.log 2>&1 || { tail -5 gpurun_out/r3r_pk_$rows.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r3r_pk_$rows.log').read().strip().splitlines()[-1])['parakeet']['streaming_1s_b64']; print('$rows', d['rtfx'], d['phases_ms'])"
done
PK_BENCH_ONLY=stream64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r_prof -o run -- python3 bench.py --parakeet-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3r_prof.log 2>&1 || { tail -5 gpurun_out/r3r_prof.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3r_prof/run_kernel_stats.csv 40 | grep -i "dec_kernel\|joint_fin"
rm -f gpurun_out/r3r_prof/run_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r_wprof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-app-latency --no-probe --no-parakeet > gpurun_out/r3r_wprof.log 2>&1 || { tail -5 gpurun_out/r3r_wprof.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3r_wprof/run_kernel_stats.csv 40 | grep -i "ln_kernel\|ln_pend\|q64\|gemm256"
rm -f gpurun_out/r3r_wprof/run_kernel_trace.csv
