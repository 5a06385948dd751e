"""whisper_full restated on the CPU oracle: the timestamp / no-timestamp greedy decoding rules,
the per-decoder bookkeeping and the seek-driven window loop with segments.

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): the checker for the product's
spittle_amd/csrc/k_sample.hip (per-token rules, on the device) and full.cpp (window loop).

Restates whisper.cpp ~1.7.x (vendored by whisper-rs-sys 0.11.1, /root/reference/src-tauri/
Cargo.lock:8156-8174; not present here, so "parity unpinned" against whisper.cpp itself):
  * whisper_process_logits (greedy, temperature 0): suppression, timestamp pairing, initial
    timestamp bound, monotonic timestamps, the timestamp-probability-mass rule;
  * whisper_sample_token (best): first maximum; plog; tid;
  * whisper_full_with_state: decoder bookkeeping (seek_delta, result_len, failure / completion),
    whisper_sequence_score, seek loop, prompt_past, segment assembly.
Temperature sampling (fallback) draws from a device stream and is not restated; the window
loop here runs greedy decoding at temperature 0 only (temperature_inc = 0).
Each step recomputes the decoder over the whole token prefix (oracle.wo_decode_logits).  Every
window's encoder input is frames [seek, seek + 3000) of ONE log-mel of the whole input
(oracle.mel_full: whisper_pcm_to_mel's global max - 8 clamp), as whisper_full_with_state does.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import oracle as O

N_LEN_HOP = 160


@dataclass
class Params:
    no_timestamps: bool = False
    suppress_blank: bool = True
    max_initial_ts: float = 1.0
    max_tokens: int = 0
    entropy_thold: float = 2.4
    logprob_thold: float = -1.0
    n_max_text_ctx: int = 16384
    translate: bool = False
    beam_size: int = 1


@dataclass
class Step:
    tok: int
    plog: float
    tid: int
    margin: float     # smallest decision gap of this step (argmax gap, timestamp-rule gap)


@dataclass
class Window:
    steps: list = field(default_factory=list)
    has_ts: bool = False
    seek_delta: int = 3000
    result_len: int = 0
    status: int = 0   # 1 completed, 2 failed


def static_mask(n_vocab: int, sp: dict, no_timestamps_fast: bool = False, extra=()) -> np.ndarray:
    m = np.zeros(n_vocab, bool)
    for k in ("not", "sot", "nosp", "solm", "translate", "transcribe", "prev"):
        m[sp[k]] = True
    m[sp["sot"] + 1: sp["sot"] + 1 + sp["n_langs"]] = True
    for t in extra:
        m[t] = True
    return m


def pick(lg: np.ndarray, step: int, toks: list, w: Window, p: Params, sp: dict, smask: np.ndarray,
         blank: int = 220, max_initial: int = 50):
    """whisper_process_logits + whisper_sample_token (greedy) for one step."""
    eot, beg = sp["eot"], sp["beg"]
    v = lg.astype(np.float64).copy()
    mask = smask.copy()
    if step == 0 and p.suppress_blank:
        mask[eot] = mask[blank] = True
    if p.no_timestamps:
        mask[beg:] = True
    last_ts = len(toks) > 0 and toks[-1] >= beg
    pen_ts = len(toks) < 2 or toks[-2] >= beg
    if last_ts:
        if pen_ts:
            mask[beg:] = True
        else:
            mask[:eot] = True
    if step == 0 and max_initial >= 0:
        mask[beg + max_initial + 1:] = True
    if w.has_ts:
        mask[beg:beg + w.seek_delta // 2] = True
    v[mask] = -np.inf
    M = v.max()
    lse = np.log(np.exp(v[np.isfinite(v)] - M).sum()) + M
    text, ts = v[:beg], v[beg:]
    mt = text.max()
    ms = ts.max()
    margin = np.inf
    rule = False
    if np.isfinite(ms):
        tsl = np.log(np.exp(ts[np.isfinite(ts)] - ms).sum()) + ms
        rule = tsl > mt
        margin = abs(tsl - mt)
    cand = v.copy()
    if rule:
        cand[:beg] = -np.inf
    i = int(np.argmax(cand))
    srt = np.sort(cand[np.isfinite(cand)])
    if srt.size > 1:
        margin = min(margin, srt[-1] - srt[-2])
    plog = float(v[i] - lse)
    tid = i if i >= beg else (int(np.argmax(ts)) + beg if np.isfinite(ms) else 0)
    return i, plog, tid, float(margin)


def topk(lg: np.ndarray, step: int, toks: list, w: Window, p: Params, sp: dict, smask: np.ndarray, k: int,
         blank: int = 220, max_initial: int = 50):
    """beam candidates of one decoder: the k best processed logits (after the timestamp rule,
    ties: lower id) as (id, logprob, tid), plus the smallest gap around the k-th place."""
    eot, beg = sp["eot"], sp["beg"]
    v = lg.astype(np.float64).copy()
    mask = smask.copy()
    if step == 0 and p.suppress_blank:
        mask[eot] = mask[blank] = True
    if p.no_timestamps:
        mask[beg:] = True
    last_ts = len(toks) > 0 and toks[-1] >= beg
    pen_ts = len(toks) < 2 or toks[-2] >= beg
    if last_ts:
        if pen_ts:
            mask[beg:] = True
        else:
            mask[:eot] = True
    if step == 0 and max_initial >= 0:
        mask[beg + max_initial + 1:] = True
    if w.has_ts:
        mask[beg:beg + w.seek_delta // 2] = True
    v[mask] = -np.inf
    M = v.max()
    lse = np.log(np.exp(v[np.isfinite(v)] - M).sum()) + M
    mt, ms = v[:beg].max(), v[beg:].max()
    margin = np.inf
    rule = False
    if np.isfinite(ms):
        tsl = np.log(np.exp(v[beg:][np.isfinite(v[beg:])] - ms).sum()) + ms
        rule = tsl > mt
        margin = abs(tsl - mt)
    cand = v.copy()
    if rule:
        cand[:beg] = -np.inf
    order = np.lexsort((np.arange(len(cand)), -cand))[:k + 1]
    tid = int(np.argmax(v[beg:])) + beg if np.isfinite(ms) else 0
    out = [(int(i), float(v[i] - lse), int(i) if i >= beg else tid) for i in order[:k] if np.isfinite(cand[i])]
    if len(order) > k and np.isfinite(cand[order[k]]):
        margin = min(margin, cand[order[k - 1]] - cand[order[k]])
    return out, float(margin)


def bookkeep(w: Window, tok: int, i: int, seek: int, seek_end: int, p: Params, sp: dict, n_max: int) -> None:
    eot, beg = sp["eot"], sp["beg"]
    if tok > beg:
        sdn = 2 * (tok - beg)
        if w.has_ts and w.seek_delta > sdn and w.result_len < i:
            w.status = 2
            return
        w.seek_delta, w.result_len, w.has_ts = sdn, i + 1, True
    if tok == eot or (p.max_tokens > 0 and i >= p.max_tokens) or (w.has_ts and seek + w.seek_delta + 100 >= seek_end):
        if w.result_len == 0 and not p.no_timestamps:
            if seek + w.seek_delta + 100 >= seek_end:
                w.result_len = i + 1
            else:
                w.status = 2
                return
        if p.no_timestamps:
            w.result_len, w.seek_delta = i + 1, 3000
        w.status = 1
        return
    if i == n_max - 1 and (w.result_len == 0 or w.seek_delta < 1500):
        w.status = 2


def decode_window(m: O.Model, enc: np.ndarray, prompt: list, seek: int, seek_end: int, p: Params,
                  n_steps: int, blank: int = 220) -> Window:
    sp = O.special_tokens(m.dims.n_vocab)
    smask = static_mask(m.dims.n_vocab, sp)
    n_max = m.dims.n_text_ctx // 2 - 4
    w = Window()
    toks: list = []
    for i in range(n_steps):
        lg = m.logits(enc, prompt + toks)
        t, plog, tid, margin = pick(lg, i, toks, w, p, sp, smask, blank)
        w.steps.append(Step(t, plog, tid, margin))
        toks.append(t)
        bookkeep(w, t, i, seek, seek_end, p, sp, n_max)
        if w.status:
            break
    return w


def decode_window_beam(m: O.Model, enc: np.ndarray, prompt: list, seek: int, seek_end: int, p: Params,
                       n_steps: int, blank: int = 220) -> list:
    """whisper_full's beam search at temperature 0 (see spittle_amd/csrc/full.cpp run_beam):
    returns the K decoders (Windows; margin = the smallest candidate gap of the step)."""
    import copy
    sp = O.special_tokens(m.dims.n_vocab)
    smask = static_mask(m.dims.n_vocab, sp)
    n_max = m.dims.n_text_ctx // 2 - 4
    K = p.beam_size
    decs = [Window() for _ in range(K)]
    sums = [0.0] * K
    for i in range(n_steps):
        cands = []
        gap = np.inf
        for d in range(K):
            w = decs[d]
            if w.status:
                continue
            toks = [s.tok for s in w.steps]
            lg = m.logits(enc, prompt + toks)
            out, mg = topk(lg, i, toks, w, p, sp, smask, K, blank)
            gap = min(gap, mg)
            for tok, lp, tid in out:
                cands.append((d, sums[d] + lp, tok, lp, tid))
        if not cands:
            break
        cands.sort(key=lambda c: (-c[1], c[0]))
        # the cut across decoders: the distinct cumulative scores the live decoders take (step 0:
        # every decoder takes the single best, later steps skip exact repeats) and the first one
        # left out.  Exact repeats (identical decoder rows) are deduplicated by equality, which the
        # GPU reproduces bitwise; a near-tie between different scores is an uncertain decision.
        live = sum(1 for w in decs if not w.status)
        distinct = []
        for c in cands:
            if not distinct or c[1] != distinct[-1]:
                distinct.append(c[1])
            if len(distinct) > (1 if i == 0 else live):
                break
        for a, b in zip(distinct, distinct[1:]):
            gap = min(gap, a - b)
        new, new_sums, cur = list(decs), list(sums), 0
        for d in range(K):
            if decs[d].status:
                continue
            if cur >= len(cands):
                cur = 0
            c = cands[cur]
            cur += 1
            while len(cands) > cur and cands[cur][1] == c[1] and i > 0:
                cur += 1
            w = copy.deepcopy(decs[c[0]])
            w.steps.append(Step(c[2], c[3], c[4], gap))
            new[d], new_sums[d] = w, c[1]
        for d in range(K):
            if decs[d].status == 0:
                bookkeep(new[d], new[d].steps[-1].tok, i, seek, seek_end, p, sp, n_max)
        decs, sums = new, new_sums
        if all(w.status for w in decs):
            break
    return decs


def n_len_org(n: int) -> int:
    return 1 + int((n + 200 - 400) / N_LEN_HOP)  # C integer division (toward zero)


def transcribe(m: O.Model, pcm: np.ndarray, p: Params, prompt=(), lang_tok: int = -1):
    """whisper_full at temperature 0 without fallback.  Returns (windows, segments, tokens, kept):
    windows = [(seek, Window)], segments = [(t0, t1, text, i0, n)] with text the "[id]" spelling,
    tokens = every window's result tokens, kept = their Steps (plog, tid, margin)."""
    sp = O.special_tokens(m.dims.n_vocab)
    eot, beg = sp["eot"], sp["beg"]
    multi = sp["n_langs"] > 0
    no_ts = p.no_timestamps or (m.dims.n_dec == 2 and m.dims.n_vocab != 51866)
    pp = Params(**{**p.__dict__, "no_timestamps": no_ts})
    init = [sp["sot"]]
    if multi:
        init += [lang_tok if lang_tok >= 0 else sp["sot"] + 1, sp["translate"] if p.translate else sp["transcribe"]]
    if no_ts:
        init.append(sp["not"])
    n_max = m.dims.n_text_ctx // 2 - 4
    seek, seek_end = 0, n_len_org(len(pcm))
    past = list(prompt)
    # whisper_pcm_to_mel: one log-mel of the whole input (global max), sliced per window
    mel_all = O.mel_full(pcm, m.dims.n_mels)
    wins, segs, all_toks, kept = [], [], [], []
    while seek + 100 < seek_end:
        if seek > 0 and seek + 500 >= seek_end:
            past = []
        pf = []
        if past and p.n_max_text_ctx > 0:
            n_take = min(p.n_max_text_ctx, m.dims.n_text_ctx // 2, len(past))
            pf = [sp["prev"]] + past[len(past) - n_take:]
        enc = m.encode(O.mel_window(mel_all, seek))
        steps = min(n_max, m.dims.n_text_ctx + 1 - len(pf) - len(init))
        if p.beam_size > 1:
            decs = decode_window_beam(m, enc, pf + init, seek, seek_end, pp, steps)
        else:
            decs = [decode_window(m, enc, pf + init, seek, seek_end, pp, steps)]

        def scored(w):  # whisper_sequence_score + the entropy check: (failed, score)
            if w.status == 2:
                return True, -np.inf
            rl = w.result_len
            if rl == 0:
                return False, -np.inf
            toks_ = [s.tok for s in w.steps]
            cnt = {}
            for t in toks_[max(0, rl - 32):rl]:
                cnt[t] = cnt.get(t, 0) + 1
            n = sum(cnt.values())
            ent = -sum(c / n * np.log(c / n) for c in cnt.values())
            if rl > 32 and ent < p.entropy_thold:
                return True, -np.inf
            return False, sum(s.plog for s in w.steps[:rl]) / rl

        best, best_score = 0, -np.inf
        flags = [scored(w) for w in decs]
        for d, (f, sc) in enumerate(flags):
            if not f and best_score < sc:
                best, best_score = d, sc
        w = decs[best]
        failed = flags[best][0]
        wins.append((seek, w))
        toks = [s.tok for s in w.steps]
        tids = [s.tid for s in w.steps]
        n_keep = len(toks) if failed else min(w.result_len, len(toks))
        toks, tids = toks[:n_keep], tids[:n_keep]
        base = len(all_toks)
        all_toks += toks
        kept += w.steps[:n_keep]
        past = (pf[1:] if pf else []) + [s.tok for s in w.steps[:w.result_len]]
        if toks:
            i0, t0, text, i = 0, seek + 2 * (tids[0] - beg), "", 0
            while i < len(toks):
                if toks[i] < eot:
                    text += f"[{toks[i]}]"
                if toks[i] > beg:
                    t1 = seek + 2 * (tids[i] - beg)
                    if text:
                        segs.append((t0, t1, text, base + i0, i - i0 + 1))
                    text = ""
                    while i < len(toks) and toks[i] > beg:
                        i += 1
                    i -= 1
                    t0, i0 = t1, i + 1
                i += 1
            if text:
                segs.append((t0, seek + w.seek_delta, text, base + i0, len(toks) - i0))
        seek += w.seek_delta if w.seek_delta > 0 else 3000
    return wins, segs, all_toks, kept
