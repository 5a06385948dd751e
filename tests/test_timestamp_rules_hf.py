"""Partial pinning of the whisper_full timestamp rules (oracle/whisper_full.py pick, restated
from whisper.cpp whisper_process_logits; k_sample.hip implements the same rules on the device)
against an independent implementation available offline: HF transformers'
WhisperTimeStampLogitsProcessor (after openai/whisper decoding.py ApplyTimestampRules).

The two agree on: timestamps in pairs, the timestamp-probability-mass rule, [notimestamps]
suppression, and no timestamp below the last one.  Known, documented differences (not checked):
HF forces a timestamp as the first token (whisper.cpp does not: only max_initial_ts), and after
a text token HF also forbids repeating the last timestamp (whisper.cpp masks below it only).
So: steps >= 1, and the last timestamp id itself is excluded from the comparison when the last
token is text.  Random logits (numpy seed), random token histories; CPU only."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import whisper_full as W

torch = pytest.importorskip("torch")
lp = pytest.importorskip("transformers.generation.logits_process")


class _Cfg:
    def __init__(self, sp):
        self.no_timestamps_token_id = sp["not"]
        self.eos_token_id = sp["eot"]
        self.bos_token_id = sp["sot"]
        self.max_initial_timestamp_index = 50


def _oracle_mask(lg, toks, sp, n_vocab):
    """the oracle's candidate set at step len(toks) (after every rule, incl. the mass rule)"""
    w = W.Window()
    for i, t in enumerate(toks):  # replay the bookkeeping that sets has_ts / seek_delta
        if t > sp["beg"]:
            w.has_ts, w.seek_delta = True, 2 * (t - sp["beg"])
    smask = np.zeros(n_vocab, bool)
    smask[sp["not"]] = True
    p = W.Params(suppress_blank=False)
    eot, beg = sp["eot"], sp["beg"]
    v = lg.astype(np.float64).copy()
    mask = smask.copy()
    last_ts = len(toks) > 0 and toks[-1] >= beg
    pen_ts = len(toks) < 2 or toks[-2] >= beg
    if last_ts:
        if pen_ts:
            mask[beg:] = True
        else:
            mask[:eot] = True
    if w.has_ts:
        mask[beg:beg + w.seek_delta // 2] = True
    v[mask] = -np.inf
    # cross-check against pick(): the chosen token is the argmax of this candidate set
    M = v.max()
    lse = np.log(np.exp(v[np.isfinite(v)] - M).sum()) + M
    ts = v[beg:]
    if np.isfinite(ts.max()):
        tsl = np.log(np.exp(ts[np.isfinite(ts)] - ts.max()).sum()) + ts.max()
        if tsl > v[:beg].max():
            v[:beg] = -np.inf
    i, _, _, _ = W.pick(lg, len(toks), toks, w, p, sp, smask, max_initial=-1)
    assert i == int(np.argmax(v))
    return np.isfinite(v), lse


@pytest.mark.parametrize("case", range(40))
def test_rules_match_hf(case):
    rng = np.random.default_rng(500 + case)
    n_vocab = 51864
    sp = O.special_tokens(n_vocab)
    beg, eot = sp["beg"], sp["eot"]
    # a history of 1..6 tokens mixing text and increasing timestamps, ending in either kind
    n = int(rng.integers(1, 7))
    toks, last_ts_id = [], beg
    for _ in range(n):
        if rng.random() < 0.5:
            last_ts_id = int(min(n_vocab - 1, last_ts_id + rng.integers(1, 80)))
            toks.append(last_ts_id)
        else:
            toks.append(int(rng.integers(0, eot)))
    lg = (rng.standard_normal(n_vocab) * 2.0).astype(np.float32)
    lg[beg:] += float(rng.uniform(-3, 3))  # vary the timestamp mass
    ours, _ = _oracle_mask(lg, toks, sp, n_vocab)
    proc = lp.WhisperTimeStampLogitsProcessor(_Cfg(sp), begin_index=1)
    ids = torch.tensor([[sp["sot"]] + toks])
    hf = proc(ids, torch.tensor(lg[None, :]).clone())[0].numpy()
    theirs = np.isfinite(hf)
    if not (len(toks) and toks[-1] >= beg):  # last token is text: HF also masks the last timestamp itself
        ts_hist = [t for t in toks if t >= beg]
        if ts_hist:
            theirs[ts_hist[-1]] = ours[ts_hist[-1]]
    assert np.array_equal(ours, theirs), (toks, np.flatnonzero(ours != theirs)[:10])
