"""One line per bench log: RTFx, C3 decode pass, C2 RTFx and pass (experiment summaries)."""
import json
import sys

for f in sys.argv[1:]:
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no bench line")
        continue
    d = json.loads(lines[-1])
    c2 = d.get("whisper_small_f32_b1") or {}
    print(f"{f}: RTFx {d['value']} decode_ms {d['phases_ms']['decode_ms']} "
          f"pass_ms {d['rooflines']['decode_pass']['ms_per_pass']} enc_ms {d['phases_ms']['encoder_ms']} "
          f"C2 {c2.get('rtfx')} C2_pass {(c2.get('rooflines') or {}).get('decode_pass', {}).get('ms_per_pass')}")
