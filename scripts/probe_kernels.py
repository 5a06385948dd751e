"""GPU box, developer A/B: one large-v3 bf16 B=8 fast-path call, then the engine's kernel probes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

torch.cuda.init()
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
from spittle_amd.synth import synth_audio

e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8))
e.load_model("synthetic:large-v3")
p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=16)
pcm = [synth_audio(i) for i in range(8)]
e.transcribe_batch(pcm, p)
out = {k: e.probe(k, 20) for k in sys.argv[1:]}
out["encoder_ms"] = e.timings()["encoder_ms"]
print(json.dumps(out))
