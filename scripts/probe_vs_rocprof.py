"""Agreement of bench.py's HIP-event kernel probes with rocprofv3: one bench run
under rocprofv3 --kernel-trace (SPT_ENC_GROUPS=1, so each encoder kernel is one full-batch launch),
then for every probed kernel: the probe's average (the bench line's `kernels`), rocprofv3's average
over the same launches, and rocprofv3's average over the timed calls' launches.  Each encoder probe
runs encoder layer 0 `iters` times (every kernel of the layer, events around its own), fc1's probe
first, then the attention's: in the trace the last 2 x iters dispatches of each kernel are the two
probes' runs, fc1's own block the first of them, the attention's the second.
usage: probe_vs_rocprof.py RESULTS_DB BENCH_LINE_JSON [ITERS]"""
import json
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
line = json.loads([ln for ln in open(sys.argv[2]).read().splitlines() if ln.startswith("{")][-1])  # (rocprofv3 prints after it)
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 50
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
# encoder probes (kind 4 / 5): `iters` runs of encoder layer 0 in sequence after the timed calls; the
# kernel names: fc1 with the LayerNorm fold (EPI_BIAS_GELU | EPI_LNF = 17) or without (1)
PAT = {"enc_fc1_gemm": ["gemm256_kernel<17,", "gemm256_kernel<1,"], "enc_attn": ["attn_bf16_q64_kernel<"]}
out = {}
for k, pats in PAT.items():
    if k not in (line.get("kernels") or {}):
        continue
    rows = []
    for pat in pats:
        rows = db.execute(f"select start, end from kernels where {name} like ? order by start", ("%" + pat + "%",)).fetchall()
        if rows:
            break
    if not rows:
        continue
    d = [(e - s) / 1e3 for s, e in rows]
    probe = line["kernels"][k]["avg_us"]
    blk = 0 if k == "enc_attn" else 1  # blocks of `iters` from the end: attention probe last
    last = d[len(d) - (blk + 1) * iters:len(d) - blk * iters]
    body = d[:len(d) - 2 * iters]
    out[k] = {"probe_avg_us": probe, "rocprof_same_launches_avg_us": round(sum(last) / len(last), 3),
              "rocprof_timed_calls_avg_us": round(sum(body) / len(body), 3), "dispatches": len(d),
              "probe_vs_same_launches_pct": round(100.0 * (probe / (sum(last) / len(last)) - 1.0), 2),
              "probe_vs_timed_calls_pct": round(100.0 * (probe / (sum(body) / len(body)) - 1.0), 2)}
print(json.dumps(out, indent=1))
