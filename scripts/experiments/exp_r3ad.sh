# r3 final: rocprofv3 kernel stats of the Parakeet C5 pass (64 x 1 s windows) and of the offline pass
# on the final tree
export TMPDIR=/tmp
mkdir -p gpurun_out
PK_BENCH_ONLY=stream64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ad_s -o run -- python3 bench.py --parakeet-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3ad_s.log 2>&1 || { tail -5 gpurun_out/r3ad_s.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3ad_s/run_kernel_stats.csv 25 > gpurun_out/r3ad_stream64_top.txt
rm -f gpurun_out/r3ad_s/run_kernel_trace.csv
PK_BENCH_ONLY=offline timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ad_o -o run -- python3 bench.py --parakeet-only --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3ad_o.log 2>&1 || { tail -5 gpurun_out/r3ad_o.log; exit 1; }
python3 profiles/summarize.py gpurun_out/r3ad_o/run_kernel_stats.csv 25 > gpurun_out/r3ad_offline_top.txt
rm -f gpurun_out/r3ad_o/run_kernel_trace.csv
echo done
