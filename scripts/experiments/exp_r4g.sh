# r4g: the beam-5 shared-window case under two builds of the attention schedule
# (v1: rolled loop only; v2: straight-line schedule without the early exit; v3: v2 without the query-loop break)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 2 3; do
  DIAG_LIB=spittle_amd/libspittle_hip_v$v.so timeout -k 10 200 python3 -u scripts/experiments/diag_beam.py > gpurun_out/r4g_$v.log 2>&1 || { tail -20 gpurun_out/r4g_$v.log; exit 1; }
done
grep -h -E "^(env|oracle)" gpurun_out/r4g_*.log
