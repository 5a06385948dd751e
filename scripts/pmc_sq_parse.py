"""Mean per-launch SQ counters of the encoder kernels from scripts/pmc_sq.sh's two passes."""
import csv
import glob
import re
from collections import defaultdict

PAT = {"attn": r"attn_bf16", "gemm_fc1": r"gemm256_kernel<1", "gemm_qkv": r"gemm256_kernel<0", "gemm_resid": r"gemm256_kernel<3",
       "ln": r"ln_kernel"}
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/sq_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k, p in PAT.items():
            if re.search(p, r.get("Kernel_Name", "")):
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
