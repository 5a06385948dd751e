"""GPU checks at BASELINE's benchmark configuration itself (C3: whisper-large-v3, all 32 + 32
layers, bf16, batch 8 x 30 s, greedy "en", no timestamps), where the oracle is too slow for a
token-for-token run over the whole batch.

* Size-independent properties over the full batch, bitwise: a window's result does not depend
  on its batch neighbours; the device-resident fast path (what bench.py times) and the host-PCM
  path agree; a second run repeats the first.
* One window against the CPU oracle (fp32 C restatement, full depth): teacher-forced on the
  oracle's tokens.  Tolerance: bf16 activations at GEMM inputs through 64 layers -> top-1
  logit within 0.1 (measured r1: max 0.030, mean 0.012 over 12 steps), and the greedy token
  equal wherever the oracle's top-1/top-2 gap > 0.2.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 1234
SPEC = "synthetic:large-v3"
B = 8


@pytest.fixture(scope="module")
def eng():
    import torch
    from spittle_amd import WhisperEngine, WhisperModelParams
    # torch's bundled HIP runtime initialises before the library's (the order bench.py uses)
    torch.zeros(1, device="cuda:0")
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=B, seed=SEED))
    e.load_model(SPEC)
    yield e
    e.unload_model()


def _params(**kw):
    from spittle_amd import WhisperInferenceParams
    return WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, **kw)


def test_fullsize_batch_properties(eng):
    import torch
    n = 32
    xs = [O.synth_audio(i) for i in range(B)]  # bench.py's chunks (BASELINE.md §3 seeds)
    p = _params(max_new_tokens=n)
    host = eng.transcribe_batch(xs, p)
    assert all(len(r.tokens) == n for r in host)
    # device-resident PCM (the bench path)
    pcm = torch.from_numpy(np.stack(xs)).to("cuda:0")
    dev = eng.transcribe_batch_device(pcm.data_ptr(), pcm.shape[1], [pcm.shape[1]] * B, p)
    for a, b in zip(host, dev):
        assert a.tokens == b.tokens
        assert np.array_equal(a.top1, b.top1) and np.array_equal(a.top2, b.top2)
    # batch invariance: windows 0 and 5 alone
    for i in (0, 5):
        alone = eng.transcribe_samples(xs[i], p)
        assert alone.tokens == host[i].tokens
        assert np.array_equal(alone.top1, host[i].top1)
    # repeatability
    again = eng.transcribe_batch(xs, p)
    for a, b in zip(host, again):
        assert a.tokens == b.tokens and np.array_equal(a.top1, b.top1)
    # the 8 windows are different inputs: not all results alike
    assert len({tuple(r.tokens) for r in host}) > 1


def test_fullsize_teacher_forced_vs_oracle(eng):
    n = 24
    om = O.Model(O.dims_for("large-v3"), SEED, O.W_BF16)
    x = O.synth_audio(0)
    enc = om.encode(O.mel(x, om.dims.n_mels))
    tk, t1, t2 = om.decode(enc, O.default_prompt(om.dims.n_vocab), n, O.SUPPRESS_BLANK | O.NO_TIMESTAMPS | O.IGNORE_EOT)
    del om
    forced = np.asarray(tk, np.int32)[None, :]
    r = eng.transcribe_batch([x], _params(max_new_tokens=n, forced_tokens=forced))[0]
    got = np.array(r.tokens)
    d = np.abs(np.asarray(r.top1) - t1)
    print("full-depth teacher-forced: max |top1 diff| %.4f, mean %.4f, min gap %.3f" % (d.max(), d.mean(), (t1 - t2).min()))
    assert d.max() < 0.1, d
    clear = (t1 - t2) > 0.2
    assert (got[clear] == np.asarray(tk)[clear]).all()


# ---------------------------------------------------------------- free-running, whole batch
# The benchmark batch itself (bench.py's 8 windows, seeds 1000-1007), greedy for the full 128
# steps on both sides, no teacher forcing: the HIP path's tokens must equal the fp32 oracle's
# (bf16-rounded weights, the same synthetic model) up to the oracle's first step whose
# top-1/top-2 gap is below FREE_GAP (a decision bf16 activations may flip), with the top-1
# logit within FREE_TOL on that matched prefix.  Per-window agreement is printed and written to
# gpurun_out/fullsize_parity.json (BASELINE.md §4's token-parity column).
FREE_STEPS = 128
FREE_GAP = 0.2
FREE_TOL = 0.1


@pytest.fixture(scope="module")
def free_run(eng):
    xs = [O.synth_audio(i) for i in range(B)]
    return xs, eng.transcribe_batch(xs, _params(max_new_tokens=FREE_STEPS))


_SUMMARY = {}


@pytest.mark.parametrize("w", range(B))
def test_fullsize_free_running_vs_oracle(free_run, w):
    import json
    xs, res = free_run
    om = O.Model(O.dims_for("large-v3"), SEED, O.W_BF16)
    enc = om.encode(O.mel(xs[w], om.dims.n_mels))
    tk, t1, t2 = om.decode(enc, O.default_prompt(om.dims.n_vocab), FREE_STEPS,
                           O.SUPPRESS_BLANK | O.NO_TIMESTAMPS | O.IGNORE_EOT)
    del om
    got = np.array(res[w].tokens)
    assert len(got) == FREE_STEPS
    tk = np.asarray(tk)
    same = got == tk
    agree = FREE_STEPS if same.all() else int(np.argmin(same))       # identical leading tokens
    gap = t1 - t2
    unsure = np.nonzero(gap < FREE_GAP)[0]
    first_unsure = int(unsure[0]) if unsure.size else FREE_STEPS
    k = min(agree, FREE_STEPS)
    d = np.abs(np.asarray(res[w].top1)[:k] - t1[:k])
    row = {"window": w, "agree_steps": agree, "first_small_gap": first_unsure,
           "max_dtop1_matched": float(d.max()) if k else None, "mean_dtop1_matched": float(d.mean()) if k else None,
           "min_gap": float(gap.min())}
    print("free-running window", json.dumps(row))
    _SUMMARY[w] = row
    if len(_SUMMARY) == B:
        os.makedirs("gpurun_out", exist_ok=True)
        tot = sum(r["agree_steps"] for r in _SUMMARY.values())
        with open(os.path.join("gpurun_out", "fullsize_parity.json"), "w") as f:
            json.dump({"steps": FREE_STEPS, "gap": FREE_GAP, "tol": FREE_TOL, "agreement_rate": tot / (B * FREE_STEPS),
                       "windows": [_SUMMARY[i] for i in range(B)]}, f, indent=1)
    # tokens equal up to the oracle's first uncertain decision ...
    assert agree >= first_unsure, row
    # ... and the logits close on everything that matched
    assert k == 0 or d.max() < FREE_TOL, row


def test_repeatable_under_uneven_load(eng):
    """Bitwise repeatability of the shipped kernels (the LDS-DMA staged GEMMs and attention, the
    decoder's flash-decoding and GEMVs) while a concurrent stream perturbs their timing: a hazard
    in an LDS ring or a cross-workgroup hand-off shows as a run-to-run difference under uneven
    load, not on an idle chip (MI355X_MICROARCH.md § visibility).  r3's dropped attention variant B
    differed by 1 bf16 ulp in 1 of 3 runs (root cause there); this checks that no
    shipped kernel does: 8 runs of the encoder at full depth and of the whole bench batch, half of
    them beside a side-stream copy loop."""
    import torch
    xs = [O.synth_audio(i) for i in range(B)]
    mel = O.mel(xs[3], 128)
    p = _params(max_new_tokens=16)
    ref_enc = eng.debug_encode(mel)
    ref = eng.transcribe_batch(xs, p)
    side = torch.cuda.Stream()
    a = torch.empty(64 << 20, dtype=torch.float32, device="cuda:0")
    b = torch.empty_like(a)
    for run in range(8):
        if run % 2:
            with torch.cuda.stream(side):  # ~25 GB of copies queued beside the engine's streams
                for _ in range(48):
                    b.copy_(a)
        enc = eng.debug_encode(mel)
        res = eng.transcribe_batch(xs, p)
        assert np.array_equal(enc, ref_enc), (run, float(np.abs(enc - ref_enc).max()))
        for x, y in zip(ref, res):
            assert x.tokens == y.tokens and np.array_equal(x.top1, y.top1) and np.array_equal(x.top2, y.top2), run
        side.synchronize()
