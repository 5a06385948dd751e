"""Diagnose the persistent decoder pass against the layered kernels on the bench shape
(B=8, greedy, 128 steps), growing the decoder depth; prints the first divergence, any
NaN sentinel (-2 tokens) and the per-pass time of both paths."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

B, N = 8, 128
xs = [synth_audio(i) for i in range(B)]
p = WhisperInferenceParams(language="en", ignore_eot=True, max_new_tokens=N)
for spec in (sys.argv[1:] or ["synthetic:large-v3:enc=1:dec=4", "synthetic:large-v3:enc=1:dec=32",
                             "synthetic:large-v3"]):
    dec = spec
    out = {}
    for persist in ("1", "0"):
        os.environ["SPT_PERSIST"] = persist
        e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=B, seed=1234))
        e.load_model(spec)
        try:
            r = e.transcribe_batch(xs, p)
            t0 = time.perf_counter()
            r = e.transcribe_batch(xs, p)
            dt = time.perf_counter() - t0
            tm = e.timings()
            pr = e.probe("dec_pass", 5)["avg_us"] if persist == "1" else None
            out[persist] = (np.array([x.tokens for x in r]), np.array([x.top1 for x in r]), dt, tm["decode_ms"], pr)
        except Exception as ex:  # noqa: BLE001
            print(f"dec={dec} persist={persist}: {type(ex).__name__}: {ex}", flush=True)
            out[persist] = None
        e.unload_model()
    if out["1"] is None or out["0"] is None:
        continue
    tp, vp, dtp, dmp, pr = out["1"]
    tl, vl, dtl, dml, _ = out["0"]
    bad = int((tp == -2).sum())
    diff = np.argwhere(tp != tl)
    first = diff[0].tolist() if len(diff) else None
    fin = np.isfinite(vp).all()
    dv = np.nanmax(np.abs(vp - vl)) if fin else float("nan")
    print(f"dec={dec}: nan-sentinels={bad} finite={fin} first-token-diff={first} n-diff={len(diff)} "
          f"max|top1 diff|={dv:.4f} decode_ms persist={dmp:.1f} layered={dml:.1f} pass_probe_us={pr}",
          flush=True)
