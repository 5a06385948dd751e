import sys, numpy as np
sys.path.insert(0, '.')
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
from spittle_amd.synth import synth_audio
p = WhisperInferenceParams(language="en", ignore_eot=True, max_new_tokens=6)
for mb, B in ((16, 8), (8, 7), (8, 8), (16, 16), (12, 8), (8, 1)):
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=mb)); e.load_model("synthetic:tiny.en")
    xs = [synth_audio(i) for i in range(B)]
    res = e.transcribe_batch(xs, p)
    print("max_batch", mb, "B", B, [r.tokens[:3] for r in res[:3]], flush=True)
    e.unload_model()
