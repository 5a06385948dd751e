# r4r: the one-row A_ATTN prologue back to one element per round (bench line), then one SQ counter
# pass over a beam call (issue / wait breakdown of beam_topk_kernel)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4r
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parakeet --no-turbo > gpurun_out/r4r/bench.log 2>&1 || { tail -5 gpurun_out/r4r/bench.log; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4r/bench.log').read().strip().splitlines()[-1]); a=d['app_call_latency_b1']
print('rtfx', d['value'], 'pass', d['rooflines']['decode_pass']['ms_per_pass'], {k: (a[k]['decode_ms_per_pass'], a[k]['ms']) for k in a})"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
MODE=beam CALLS=0 timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/r4r/sq -o run -- python3 -u scripts/experiments/prof_r4d.py > gpurun_out/r4r/sq.log 2>&1 || { grep -v "^    @" gpurun_out/r4r/sq.log | tail -10; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r4r/sq/**/*counter_collection.csv', recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f[0])):
    k = row.get('Kernel_Name', '')
    for key in ('beam_topk', 'finalize_ts', 'attn_part_merge', 'cross_attn_vw'):
        if key in k:
            agg[key][row['Counter_Name']].append(float(row['Counter_Value']))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
rm -rf gpurun_out/r4r/sq
