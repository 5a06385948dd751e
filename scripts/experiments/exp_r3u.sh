# r3 s2: encoder attention with the V tile swizzled too (SPT_ATTN_SWZ=3: the transposed V reads of
# keys k and k + 2 on different slots) vs the K-only swizzle (1); in-situ probe, large-v3 B = 8,
# interleaved, then parity of the encoder under SWZ=3 and an LDS bank-conflict counter pass each
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 3 1 3; do
  SPT_ATTN_SWZ=$v timeout -k 10 200 python3 scripts/probe_kernels.py enc_attn > gpurun_out/probe_r3u.log 2>&1 || { echo "probe failed: $v"; tail -5 gpurun_out/probe_r3u.log; exit 1; }
  echo "SWZ=$v $(tail -1 gpurun_out/probe_r3u.log)"
done
SPT_ATTN_SWZ=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "encoder or bf16" --timeout 300 --timeout-method thread > gpurun_out/r3u_tests.log 2>&1 || { tail -20 gpurun_out/r3u_tests.log; exit 1; }
tail -1 gpurun_out/r3u_tests.log
for v in 1 3; do
  SPT_ATTN_SWZ=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r3u_pmc$v -o run -- python3 scripts/probe_kernels.py enc_attn > gpurun_out/r3u_pmc$v.log 2>&1 || { echo "pmc failed $v"; tail -5 gpurun_out/r3u_pmc$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/r3u_pmc{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(list)
for fn in f:
    for r in csv.DictReader(open(fn)):
        if "q64" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("SWZ", sys.argv[1], {k: sum(v) / len(v) for k, v in acc.items()})
PY
  rm -rf gpurun_out/r3u_pmc$v/*/*kernel_trace.csv
done
