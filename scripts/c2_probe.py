"""GPU box, C2 traffic (BASELINE.json configs[1]: Whisper-small f32, B = 1, greedy fast path): two
calls on the same 30 s chunk, N_LO and N_HI decode steps, each preceded by a torch marker kernel, so
scripts/c2_pmc_parse.py can sum a PMC counter over each call's dispatches; (HI - LO) / (N_HI - N_LO)
is one decoder pass's traffic with the encoder, cross K/V and prompt pass cancelled out.  Run under
rocprofv3 --pmc (scripts/c2_pmc.sh) or plain (prints the calls' phase times)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

N_LO, N_HI = 8, 40
e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=1))
e.load_model("synthetic:small")
x = synth_audio(0)
mark = torch.zeros(1, device="cuda")


def call(n):
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                               max_new_tokens=n)
    e.transcribe_samples(x, p)
    return e.timings()


call(N_LO), call(N_HI)  # warm (graphs captured)
out = {}
for n in (N_LO, N_HI):
    mark.add_(1.0)  # marker dispatch (elementwise add kernel) ahead of the call
    torch.cuda.synchronize()
    out[n] = call(n)
mark.add_(1.0)
torch.cuda.synchronize()
print(json.dumps({"n_lo": N_LO, "n_hi": N_HI, "timings": out}))
e.unload_model()
