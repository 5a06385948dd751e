"""Per-kernel effective clock from scripts/pmc_clock.sh: GRBM_GUI_ACTIVE / 8 XCDs / duration, joined
with the kernel trace by dispatch id (durations from the counter CSV's own timestamps if present)."""
import csv
import glob
import re
from collections import defaultdict

PAT = {"attn": r"attn_bf16", "gemm_fc1": r"gemm256_kernel<1", "gemm_qkv": r"gemm256_kernel<0",
       "gemm_resid": r"gemm256_kernel<3", "ln": r"ln_kernel"}
dur = {}
for f in glob.glob("gpurun_out/clk/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
vals = defaultdict(list)
for f in glob.glob("gpurun_out/clk/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
            continue
        did = r.get("Dispatch_Id")
        t = dur.get(did)
        if t is None and r.get("End_Timestamp"):
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        if not t:
            continue
        for k, p in PAT.items():
            if re.search(p, r.get("Kernel_Name", "")):
                vals[k].append((float(r["Counter_Value"]) / 8 / t / 1e9, t * 1e6))
for k, v in vals.items():
    ghz = sorted(x[0] for x in v)
    us = sorted(x[1] for x in v)
    print(f"{k:10s} n={len(v):3d}  effective clock median {ghz[len(ghz) // 2]:.3f} GHz (min {ghz[0]:.3f}, max {ghz[-1]:.3f})"
          f"  duration median {us[len(us) // 2]:.1f} us")
