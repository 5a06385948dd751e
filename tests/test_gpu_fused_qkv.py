"""The fused decode-step kernel (LN1 + QKV projection + self K/V append + self-attention in one
launch, `qkv_attn_kernel` in k_dec.hip) against the two-launch path it replaces
(`gemv<GV_QKV_CACHE, A_LN>` + `self_attn_kernel`), selected per context by SPT_FUSED_QKV.

The fused kernel repeats the pair's arithmetic operation for operation, so the bar is bitwise:
tokens, top-1 and top-2 logits equal over every decode step.  Batch sizes 8 (the bench's, the
XCD-grouped block map), 3 and 1 (the plain block map), at large-v3 dims (d = 1280, the only
width the fused kernel serves) with 4 decoder layers.  The fused kernel is an opt-in variant
(measured slower); the default two-launch path's oracle parity is covered by
test_gpu_parity.py / test_gpu_fullsize.py, so bitwise equality carries it over.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SPEC = "synthetic:large-v3:enc=2:dec=4"
SEED = 77


def _engine(fused):
    from spittle_amd import WhisperEngine, WhisperModelParams
    old = os.environ.get("SPT_FUSED_QKV")
    os.environ["SPT_FUSED_QKV"] = "1" if fused else "0"
    try:
        e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8, seed=SEED))
        e.load_model(SPEC)
    finally:
        if old is None:
            del os.environ["SPT_FUSED_QKV"]
        else:
            os.environ["SPT_FUSED_QKV"] = old
    return e


@pytest.fixture(scope="module")
def pair():
    import torch
    torch.zeros(1, device="cuda:0")
    ef, eu = _engine(True), _engine(False)
    yield ef, eu
    ef.unload_model()
    eu.unload_model()


@pytest.mark.parametrize("nb", [8, 3, 1])
def test_fused_qkv_bitwise(pair, nb):
    from spittle_amd import WhisperInferenceParams
    ef, eu = pair
    n = 40
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                               max_new_tokens=n)
    xs = [O.synth_audio(100 + i) for i in range(nb)]
    rf = ef.transcribe_batch(xs, p)
    ru = eu.transcribe_batch(xs, p)
    for a, b in zip(rf, ru):
        assert len(a.tokens) == n
        assert a.tokens == b.tokens
        assert np.array_equal(np.asarray(a.top1), np.asarray(b.top1))
        assert np.array_equal(np.asarray(a.top2), np.asarray(b.top2))
