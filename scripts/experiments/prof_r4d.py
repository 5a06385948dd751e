"""r4d: what a 10 s beam-5 call and a B = 1 greedy call spend per kernel (run under
rocprofv3 --kernel-trace --stats; MODE=beam or MODE=b1 picks the call, CALLS the timed calls
after the warm one)."""
import os
import sys
import time

import torch  # noqa: F401  (as bench.py: rocprofv3 crashed at start-up in a process that loaded the HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

mode = os.environ.get("MODE", "beam")
e = WhisperEngine(WhisperModelParams(dtype="bf16", device=0, max_batch=8, seed=1234))
e.load_model("synthetic:large-v3")
if mode == "beam":
    p = WhisperInferenceParams(language="en", beam_size=5, temperature_inc=0.0)
    x = synth_audio(2010)[:16000 * 10]
elif mode == "full5":  # the app's default whisper_full call on 5 s (timestamps, fallback, best_of 5)
    p = WhisperInferenceParams(language="en")
    x = synth_audio(2005)[:16000 * 5]
else:
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                               max_new_tokens=128)
    x = synth_audio(2030)
e.transcribe_samples(x, p)
for _ in range(int(os.environ.get("CALLS", "2"))):
    t0 = time.perf_counter()
    r = e.transcribe_samples(x, p)
    ms = (time.perf_counter() - t0) * 1e3
    cs = e.call_stats()
    print(mode, round(ms, 2), {k: cs[k] for k in ("decoder_passes", "beam_steps", "decode_ms", "encoder_ms", "device_ms")},
          flush=True)
