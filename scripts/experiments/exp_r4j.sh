# r4j: kernel stats of a 10 s beam-5 call and of a B = 1 greedy call (3 calls each)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
for m in beam b1; do
  MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d/$m -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4d/$m.log 2>&1 || { grep -v "^    @" gpurun_out/r4d/$m.log | tail -20; exit 1; }
  grep -E "^(beam|b1) " gpurun_out/r4d/$m.log
done
