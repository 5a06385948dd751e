"""Encoder MFMA utilisation from scripts/pmc_mfma.sh's pass: per kernel class and over the whole
encoder (bf16 large-v3: the 256x256 GEMMs incl. the conv stem, flash attention, LayerNorm).

  busy_frac = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (1024 SIMDs x sum(GRBM_GUI_ACTIVE / 8))
  eff_clock = sum(GRBM_GUI_ACTIVE / 8) / sum(duration)        (MI355X_MICROARCH.md, DVFS)

busy_frac is the MFMA pipes' occupancy at the clock the chip actually ran (a 32x32x16 bf16
MFMA occupies its SIMD 32 cycles = the dense peak rate); busy_frac x eff_clock / 2.4 GHz is the
fraction of the nominal 2.5 PF peak.
"""
import csv
import glob
import json
import re
from collections import defaultdict

CLASSES = {"gemm": r"gemm256_kernel<[0-3], false", "attn": r"attn_bf16_q64_kernel", "ln": r"ln_kernel<unsigned short, 5>"}
ctr = defaultdict(dict)   # dispatch id -> counter -> value
name = {}
for f in glob.glob("gpurun_out/pmc_mfma/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name[did] = r.get("Kernel_Name", "")
        ctr[did][r["Counter_Name"]] = ctr[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
dur = {}
for f in glob.glob("gpurun_out/pmc_mfma/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[did] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
agg = defaultdict(lambda: defaultdict(float))
for did, c in ctr.items():
    for k, p in CLASSES.items():
        if re.search(p, name[did]):
            for key in ("all", k):
                a = agg[key]
                a["n"] += 1
                a["mfma_busy"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
                a["cycles"] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
                a["ns"] += dur.get(did, 0.0)
            break
out = {}
for k, a in agg.items():
    busy = a["mfma_busy"] / (1024.0 * a["cycles"]) if a["cycles"] else None
    clk = a["cycles"] / a["ns"] if a["ns"] else None  # GHz
    out[k] = {"dispatches": int(a["n"]), "mfma_busy_frac": busy, "eff_clock_ghz": clk,
              "frac_of_nominal_peak": busy * clk / 2.4 if busy and clk else None, "ms": a["ns"] / 1e6}
out["note"] = ("SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8); one bench step after one "
               "warm-up (both counted), SPT_NO_GRAPH=1, PMC-instrumented run (clock reads lower than unprofiled)")
json.dump(out, open("profiles/r2/pmc_encoder_mfma.json", "w"), indent=1)
print(json.dumps(out, indent=1))
