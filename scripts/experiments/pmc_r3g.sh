#!/bin/bash
# GPU box: SQ counters of the 128 x 128 and 256 x 256 GEMMs at the Parakeet streaming FF1 shape
# (M = 832, N = 4096, K = 1024, f16, swish epilogue), one counter pass per run
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pg_$i -o run -- spittle_amd/ubench gemm 832 4096 1024 5 2 > gpurun_out/pg_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pg_$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/pg_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        k = "nt128" if "gemm_nt_kernel" in n else ("g256" if "gemm256" in n else None)
        if k: vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
PY
rm -rf gpurun_out/pg_1 gpurun_out/pg_2
