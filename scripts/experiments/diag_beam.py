"""r4e: the tiny f32 beam-5 case of test_beam_search[5-20-91] under the current SPT_* env: tokens
and per-window top-1 log-probabilities, and the oracle's (printed once with OR=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from oracle import oracle as O  # noqa: E402
import spittle_amd._lib as _L  # noqa: E402
if os.environ.get("DIAG_LIB"):  # A/B against another build of the library
    _L.LIB_PATH = os.path.abspath(os.environ["DIAG_LIB"])
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402

SEED = 1234
e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=8, seed=SEED))
e.load_model("synthetic:tiny.en")
x = O.synth_audio(91, 20 * 16000)
for beam in (5, 3):
    r = e.transcribe_samples(x, WhisperInferenceParams(language="en", temperature_inc=0.0, max_new_tokens=16,
                                                       beam_size=beam))
    print("env", {k: v for k, v in os.environ.items() if k.startswith(("SPT_", "DIAG_"))}, "beam", beam, "tokens", list(r.tokens),
          "top1", [float(v) for v in r.top1], flush=True)
if os.environ.get("OR"):
    from oracle import whisper_full as W
    om = O.Model(O.dims_for("tiny.en"), SEED, O.W_F32)
    wins, segs, toks, kept = W.transcribe(om, x, W.Params(max_tokens=16, beam_size=5))
    print("oracle", toks, [(s.tok, round(s.plog, 6), s.margin) for _, w in wins for s in w.steps])
