"""GPU box: Whisper-small f32 B = 1 (C2) decode pass time, 128 greedy steps, three timed calls after a
capture call; B1_PKG selects another build (A/B on one box), B1_DUMP saves tokens / top-1 / top-2."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("B1_PKG"):
    sys.path.insert(0, os.path.abspath(os.environ["B1_PKG"]))
import numpy as np  # noqa: E402

from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=1))
e.load_model("synthetic:small")
p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=128)
x = synth_audio(0)
r = e.transcribe_samples(x, p)
for _ in range(3):
    r = e.transcribe_samples(x, p)
t = e.timings()
print(json.dumps({"decode_ms": t["decode_ms"], "pass_ms": t["decode_ms"] / t["n_decode_passes"], "encoder_ms": t["encoder_ms"]}))
if os.environ.get("B1_DUMP"):
    np.savez(os.environ["B1_DUMP"], tokens=np.array(r.tokens), top1=np.array(r.top1), top2=np.array(r.top2))
e.unload_model()
