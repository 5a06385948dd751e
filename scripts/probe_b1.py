"""GPU box, profiling / A/B: the app's B = 1 call shape on large-v3 bf16 (one 30 s window, greedy fast
path, 128 tokens; B1_BATCH = 8: the C3 batch), three timed calls after a capture call.
B1_DUMP=<file.npz>: the last call's tokens / top-1 / top-2 logits, for bitwise comparisons across
switches read at engine creation."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("B1_PKG"):  # import spittle_amd from another build (A/B between builds on one box)
    sys.path.insert(0, os.path.abspath(os.environ["B1_PKG"]))

if os.environ.get("B1_TORCH"):  # initialise HIP through torch first (its bundled runtime), as bench.py does
    import torch  # noqa: E402

    torch.cuda.init()
else:  # the Rust app's configuration: the library initialises HIP itself (the system runtime)
    import ctypes  # noqa: E402

    _st = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_trace.so"))
    os.makedirs("gpurun_out", exist_ok=True)
    _st.segv_trace_install(os.environ.get("B1_SEGV_OUT", "gpurun_out/segv_b1.txt").encode())

from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=int(os.environ.get("B1_MAX_BATCH", "8"))))
e.load_model("synthetic:large-v3")
if os.environ.get("B1_FULL"):  # the app's own call: whisper_full defaults (timestamps, fallback, best_of 5)
    p = WhisperInferenceParams(language="en")
else:
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=128)
x = synth_audio(1000)[: int(os.environ.get("B1_SAMPLES", "480000"))]
nb = int(os.environ.get("B1_BATCH", "1"))  # > 1: one batched call of that many chunks (C3 shape at 8)
xs = [synth_audio(1000 + i)[: len(x)] for i in range(nb)]
run = (lambda: e.transcribe_samples(x, p)) if nb == 1 else (lambda: e.transcribe_batch(xs, p))
run()
for _ in range(3):
    run()
t = e.timings()
cs = e.call_stats()
print(json.dumps({"decode_ms": t["decode_ms"], "passes": t["n_decode_passes"], "pass_ms": t["decode_ms"] / t["n_decode_passes"],
                  "pd_passes": cs["pd_passes"], "pd_fallbacks": cs["pd_fallbacks"]}))
if os.environ.get("B1_DUMP"):
    import numpy as np

    r = run()
    rs = [r] if nb == 1 else r
    np.savez(os.environ["B1_DUMP"], tokens=np.array([x.tokens for x in rs]), top1=np.array([x.top1 for x in rs]),
             top2=np.array([x.top2 for x in rs]))
e.unload_model()
