"""Persistent decoder pass vs the launch chain: per-pass and per-layer decode
time of the large-v3 bf16 model (32 decoder layers) at B = 1 (the app's call), 5 (beam / best_of
rows) and 8 (BASELINE C3), greedy fast path over 30 s windows, plus the app's beam-5 call; each
with SPT_PERSISTENT=0 (the chain) and 1, the outputs compared bitwise.

usage: python scripts/exp_persistent.py [out.json]   (GPU box)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402  (synthetic audio only)


def run(pd, out):
    os.environ["SPT_PERSISTENT"] = str(pd)
    from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8, seed=1234))
    e.load_model("synthetic:large-v3")
    L = e.info()["n_dec"]
    res = {}
    for B in (1, 5, 8):
        xs = [O.synth_audio(1000 + i) for i in range(B)]
        p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                                   max_new_tokens=128)
        e.transcribe_batch(xs, p)  # warm-up: graph capture
        per = []
        toks = None
        for _ in range(5):
            r = e.transcribe_batch(xs, p)
            t = e.timings()
            per.append(t["decode_ms"] / t["n_decode_passes"])
            toks = [(list(x.tokens), np.asarray(x.top1).tobytes()) for x in r]
        cs = e.call_stats()
        ms = float(np.median(per))
        res[f"greedy_b{B}"] = {"pass_ms": ms, "layer_us": 1000.0 * ms / L, "runs_ms": per, "pd_passes": cs["pd_passes"],
                               "pd_fallbacks": cs["pd_fallbacks"], "out": toks}
        print(f"pd={pd} B={B}: pass {ms:.4f} ms ({1000 * ms / L:.2f} us per layer incl. head share) pd_passes={cs['pd_passes']}",
              flush=True)
    x = O.synth_audio(1100, 10 * 16000)
    p = WhisperInferenceParams(language="en", temperature_inc=0.0, beam_size=5, max_new_tokens=32)
    e.transcribe_samples(x, p)
    per = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = e.transcribe_samples(x, p)
        wall = time.perf_counter() - t0
        cs = e.call_stats()
        per.append(cs["decode_ms"] / max(1, cs["decoder_passes"]))
    res["beam5_10s"] = {"pass_ms": float(np.median(per)), "runs_ms": per, "wall_s": wall, "decoder_passes": cs["decoder_passes"],
                        "pd_passes": cs["pd_passes"], "pd_fallbacks": cs["pd_fallbacks"],
                        "out": [(list(r.tokens), np.asarray(r.top1).tobytes())]}
    print(f"pd={pd} beam5 10 s: pass {np.median(per):.4f} ms pd_passes={cs['pd_passes']}", flush=True)
    e.unload_model()
    out[f"pd{pd}"] = res


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "exp_persistent.json")
    out = {}
    run(0, out)
    run(1, out)
    summary = {}
    for k in out["pd0"]:
        a, b = out["pd0"][k], out["pd1"][k]
        same = a["out"] == b["out"]
        summary[k] = {"chain_pass_ms": a["pass_ms"], "persistent_pass_ms": b["pass_ms"],
                      "ratio": b["pass_ms"] / a["pass_ms"], "bitwise_equal": same}
        if "layer_us" in a:
            summary[k].update({"chain_layer_us": a["layer_us"], "persistent_layer_us": b["layer_us"]})
        print(k, json.dumps(summary[k]), flush=True)
    for v in out.values():
        for r in v.values():
            r.pop("out", None)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump({"summary": summary, "raw": out}, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
