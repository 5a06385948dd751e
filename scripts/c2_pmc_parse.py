"""Per-pass HBM traffic of the C2 decode pass (scripts/c2_probe.py under rocprofv3 --pmc): the
counter summed over the dispatches between the first and second marker (the N_LO-step call) and
between the second and third (the N_HI-step call); their difference / (N_HI - N_LO) is one decoder
pass.  FETCH_SIZE (KiB) doubled per MI355X_MICROARCH.md §HBM; WRITE_SIZE (KiB) as is."""
import csv
import glob
import json
import sys

N_LO, N_HI = 8, 40
d = sys.argv[1]
res = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"{d}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    marks = [i for i, (_, n, _) in enumerate(rows) if "elementwise" in n.lower() or "vectorized" in n.lower()]
    marks = marks[-3:]
    lo = sum(v for _, _, v in rows[marks[0] + 1:marks[1]])
    hi = sum(v for _, _, v in rows[marks[1] + 1:marks[2]])
    per_pass = (hi - lo) / (N_HI - N_LO) * 1024.0
    kern = {}
    for _, n, v in rows[marks[1] + 1:marks[2]]:
        k = n.replace("(anonymous namespace)::", "").replace("void ", "")[:70]
        kern[k] = kern.get(k, 0.0) + v * 1024.0
    res[counter] = {"per_pass_bytes_raw": per_pass, "hi_call_top": sorted(kern.items(), key=lambda t: -t[1])[:12]}
fetch = 2 * res["FETCH_SIZE"]["per_pass_bytes_raw"]
write = res["WRITE_SIZE"]["per_pass_bytes_raw"]
out = {"config": "C2 Whisper-small f32 B=1 greedy fast path", "hbm_bytes_per_pass": fetch + write,
       "fetch_bytes_per_pass_x2": fetch, "write_bytes_per_pass": write, "method": "(40-step call - 8-step call) / 32",
       "detail": res}
json.dump(out, open("profiles/r6/pmc_c2_small_f32.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "detail"}))
