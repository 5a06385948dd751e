// full.cpp -- see full.h.
#include "full.h"

#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <stdexcept>

#include "engine.h"
#include "vocab.h"

namespace spt {

namespace {

constexpr int kHop = 160;     // samples per 10 ms frame

// whisper_n_len of an input: log_mel_spectrogram's n_len_org = 1 + (n + 200 - 400) / 160
int n_len_org(int n) { return 1 + (n + 200 - 400) / kHop; }

struct DecOut {                 // one decoder of one window
    std::vector<int> tok;       // generated tokens (until the decoder stopped)
    std::vector<float> plog, tid;
    int seek_delta = 0, result_len = 0, status = 0;  // status 1 completed, 2 failed
    bool failed = false;
    double avg = -INFINITY, score = -INFINITY;
};

// whisper_sequence_score + the entropy check of whisper_full (length_penalty = -1: the score
// is the average log-probability)
void score(DecOut& d, const FullParams& p) {
    const int rl = d.result_len;
    if (d.failed || rl == 0) return;
    double sum = 0.0;
    for (int i = 0; i < rl; ++i) sum += d.plog[i];
    d.avg = sum / rl;
    d.score = sum / rl;
    std::map<int, int> counts;
    int cnt = 0;
    for (int i = std::max(0, rl - 32); i < rl; ++i) {
        counts[d.tok[i]]++;
        cnt++;
    }
    double entropy = 0.0;
    for (const auto& kv : counts) {
        const double q = kv.second / (double)cnt;
        entropy -= q * log(q);
    }
    if (rl > 32 && entropy < p.entropy_thold) d.failed = true;
}

// one decoder's bookkeeping after token tok at step i (the kernel's rule, k_sample.hip)
void bookkeep(DecOut& d, int tok, int i, int seek, int seek_end, const FullParams& p, const Specials& sp, int n_max,
              bool& has_ts) {
    if (tok > sp.beg) {
        const int sdn = 2 * (tok - sp.beg);
        if (has_ts && d.seek_delta > sdn && d.result_len < i) { d.status = 2; return; }
        d.seek_delta = sdn;
        d.result_len = i + 1;
        has_ts = true;
    }
    if (tok == sp.eot || (p.max_tokens > 0 && i >= p.max_tokens) || (has_ts && seek + d.seek_delta + 100 >= seek_end)) {
        if (d.result_len == 0 && !p.no_timestamps) {
            if (seek + d.seek_delta + 100 >= seek_end) d.result_len = i + 1;
            else { d.status = 2; return; }
        }
        if (p.no_timestamps) { d.result_len = i + 1; d.seek_delta = 3000; }
        d.status = 1;
        return;
    }
    if (i == n_max - 1 && (d.result_len == 0 || d.seek_delta < 1500)) d.status = 2;  // repetition guard
}

// whisper_full's beam search at temperature 0 over nj utterances x K decoder rows (row j*K + d):
// each step every live decoder proposes its K best candidates (device, k_sample.hip
// beam_topk_kernel); the candidates of one utterance are ranked by cumulative log-probability
// (ties: lower decoder index), each live decoder takes the next one (from the second step on,
// skipping candidates whose sum equals the one just taken), its self-K/V row follows the source
// decoder, and the per-decoder bookkeeping runs on the new last token
void run_beam(Engine& e, const DecodeRequest& rq, int nj, int K, const std::vector<int>& seek,
              const std::vector<int>& seek_end, const FullParams& p, const Specials& sp, int n_max,
              std::vector<std::vector<DecOut>>* outs, std::vector<int>* lang) {
    const int B = nj * K;
    struct Dec {
        DecOut o;
        bool has_ts = false;
        double sum_all = 0.0;
    };
    std::vector<Dec> dec(B);
    for (Dec& d : dec) d.o.seek_delta = 3000;
    BeamCands c;
    lang->assign(B, -1);
    e.beam_begin(B, rq, &c, lang->data());
    struct Cand {
        int src;
        Dec d;
    };
    std::vector<int> src(B), tok(B), row((size_t)B * 4);
    for (int i = 0; i < rq.n_steps; ++i) {
        bool any = false;
        for (int j = 0; j < nj; ++j) {
            std::vector<Cand> cs;
            for (int dd = 0; dd < K; ++dd) {
                const int r = j * K + dd;
                const Dec& d = dec[r];
                if (d.o.status != 0) continue;
                for (int q = 0; q < K; ++q) {
                    const int id = c.id[(size_t)r * 8 + q];
                    if (id < 0) continue;
                    Cand cd{r, d};
                    cd.d.o.tok.push_back(id);
                    cd.d.o.plog.push_back(c.lp[(size_t)r * 8 + q]);
                    cd.d.o.tid.push_back((float)(id >= sp.beg ? id : c.tid[r]));
                    cd.d.sum_all += c.lp[(size_t)r * 8 + q];
                    cs.push_back(std::move(cd));
                }
            }
            std::stable_sort(cs.begin(), cs.end(), [](const Cand& a, const Cand& b) {
                if (a.d.sum_all != b.d.sum_all) return a.d.sum_all > b.d.sum_all;
                return a.src < b.src;
            });
            size_t cur = 0;
            std::vector<Dec> next(dec.begin() + j * K, dec.begin() + (j + 1) * K);
            for (int dd = 0; dd < K; ++dd) {
                const int r = j * K + dd;
                src[r] = r;
                if (dec[r].o.status != 0 || cs.empty()) continue;
                if (cur >= cs.size()) cur = 0;
                const Cand& pick = cs[cur++];
                while (cs.size() > cur && cs[cur].d.sum_all == pick.d.sum_all && i > 0) ++cur;
                next[dd] = pick.d;
                src[r] = pick.src;
            }
            for (int dd = 0; dd < K; ++dd) {
                const int r = j * K + dd;
                Dec& d = next[dd];
                if (dec[r].o.status == 0 && !cs.empty()) {
                    bookkeep(d.o, d.o.tok.back(), i, seek[r], seek_end[r], p, sp, n_max, d.has_ts);
                    if (d.o.status == 0) any = true;
                }
            }
            for (int dd = 0; dd < K; ++dd) dec[j * K + dd] = std::move(next[dd]);
        }
        if (!any || i + 1 >= rq.n_steps) break;
        for (int r = 0; r < B; ++r) {
            const DecOut& o = dec[r].o;
            const int n = (int)o.tok.size();
            tok[r] = n > 0 ? o.tok[n - 1] : sp.eot;
            row[r * 4 + 0] = n > 0 ? o.tok[n - 1] : -1;
            row[r * 4 + 1] = n > 1 ? o.tok[n - 2] : -1;
            row[r * 4 + 2] = dec[r].has_ts ? 1 : 0;
            row[r * 4 + 3] = o.seek_delta;
        }
        e.beam_next(src.data(), tok.data(), row.data(), i + 1, &c);
    }
    outs->assign(nj, std::vector<DecOut>());
    for (int j = 0; j < nj; ++j)
        for (int dd = 0; dd < K; ++dd) {
            DecOut o = dec[j * K + dd].o;
            o.failed = o.status == 2;
            (*outs)[j].push_back(std::move(o));
        }
}

}  // namespace

std::vector<int> non_speech_tokens(const Vocab& v) {
    // whisper_process_logits' list (after openai/whisper tokenizer.py non_speech_tokens)
    static const char* const kSyms[] = {
        "\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^", "_", "`", "{", "|",
        "}", "~", "「", "」", "『", "』", "<<", ">>", "<<<", ">>>", "--", "---", "-(", "-[", "('",
        "(\"", "((", "))", "(((", ")))", "[[", "]]", "{{", "}}", "♪♪", "♪♪♪", "♩",
        "♪", "♫", "♬", "♭", "♮", "♯"};
    std::vector<int> out;
    for (const char* s : kSyms)
        for (const std::string& t : {std::string(s), " " + std::string(s)}) {
            const int id = v.id(t);
            if (id >= 0) out.push_back(id);
        }
    for (const char* t : {" -", " '"}) {  // hyphen / quote allowed inside words only
        const int id = v.id(t);
        if (id >= 0) out.push_back(id);
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

void whisper_full_batch(Engine& e, const Vocab* vocab, const std::vector<const float*>& pcm,
                        const std::vector<int>& n, const FullParams& p_in, const std::vector<int>& prompt, int lang_tok,
                        std::vector<FullResult>* out) {
    const ModelDims& dm = e.dims();
    const Specials sp = specials_for(dm.n_vocab);
    const int U = (int)pcm.size();
    out->assign(U, FullResult());
    FullParams p = p_in;
    // first-release distilled models (2 decoder layers, not large-v3's vocabulary) need
    // [notimestamps] (whisper_full forces it)
    if (dm.n_dec == 2 && dm.n_vocab != 51866) p.no_timestamps = true;
    std::vector<float> temps;
    if (p.temperature_inc > 0.0f)
        for (float t = p.temperature; t < 1.0f + 1e-6f; t += p.temperature_inc) temps.push_back(t);
    else
        temps.push_back(p.temperature);
    const bool multi = sp.n_langs > 0;
    std::vector<int> prompt_init = {sp.sot};
    if (multi) {
        prompt_init.push_back(sp.sot + 1);  // placeholder: each sequence's language token
        prompt_init.push_back(p.translate ? sp.translate : sp.transcribe);
    }
    if (p.no_timestamps) prompt_init.push_back(sp.not_);
    const int Tq = (int)prompt_init.size();
    const int n_max = dm.n_text_ctx / 2 - 4;
    const int max_initial = p.max_initial_ts > 0.0f ? (int)lroundf(p.max_initial_ts / (30.0f / dm.n_audio_ctx)) : -1;
    const std::vector<int> nst = (p.suppress_nst && vocab) ? non_speech_tokens(*vocab) : std::vector<int>();
    const int blank = vocab ? vocab->id(" ") : 220;
    const int cap = e.max_batch();
    // best_of sampled decoders per window; more than the context's rows run in further
    // sub-batches (beam search needs its rows together: run_full rejects beam_size > max_batch)
    const int ndec_hot = std::max(1, p.best_of);

    struct Utt {
        int seek = 0, seek_end = 0;
        std::vector<int> past;
        int lang = -1;
        bool done = false;
    };
    std::vector<Utt> us(U);
    for (int u = 0; u < U; ++u) {
        us[u].seek_end = n_len_org(n[u]);
        us[u].past = prompt;  // no_context: nothing carried over from an earlier call
        us[u].lang = multi ? lang_tok : -1;
        (*out)[u].lang_tok = us[u].lang;
    }
    uint64_t call = 0;
    // one window of each utterance in `chunk` (encoded as window win_of[u]): the temperature
    // loop of whisper_full_with_state, each temperature's decoders batched over the utterances
    // SPT_NO_WINDOW_SHARE=1 (tests): each decoder row encodes its own copy of its window, as every
    // engine call did before ABI 11 -- the outputs must be bitwise the same as with shared windows
    const char* ns_env = getenv("SPT_NO_WINDOW_SHARE");
    const bool no_share = ns_env && atoi(ns_env) != 0;
    std::map<int, int> chunk_utt;  // utterance -> its index in the loaded set
    auto window_pass = [&](const std::vector<int>& chunk, const std::map<int, int>& win_of) {
        std::vector<int> pending = chunk;
        for (size_t it = 0; it < temps.size() && !pending.empty(); ++it) {
            const float t_cur = temps[it];
            const bool beam = p.beam_size > 1 && t_cur == 0.0f;  // WHISPER_SAMPLING_BEAM_SEARCH
            const int ndec = beam ? std::min(p.beam_size, cap) : t_cur > 0.0f ? ndec_hot : 1;
            const int dchunk = std::min(ndec, cap);  // decoders of one utterance per engine call
            // prompt_past conditioning: [prev] + the last min(n_max_text_ctx, n_text_ctx / 2) tokens
            std::map<int, std::vector<int>> prefix;
            for (int u : pending) {
                std::vector<int>& pf = prefix[u];
                const std::vector<int>& past = us[u].past;
                if (!past.empty() && t_cur < 0.5f && p.n_max_text_ctx > 0) {
                    const int n_take = std::min(std::min(p.n_max_text_ctx, dm.n_text_ctx / 2), (int)past.size());
                    pf.push_back(sp.prev);
                    pf.insert(pf.end(), past.end() - n_take, past.end());
                }
            }
            // batches: equal prefix lengths (one position for every row), <= cap rows
            std::map<size_t, std::vector<int>> by_len;
            for (int u : pending) by_len[prefix[u].size()].push_back(u);
            std::map<int, std::vector<DecOut>> res;
            for (auto& kv : by_len) {
                const std::vector<int>& grp = kv.second;
                const int P = (int)kv.first;
                // a beam call decodes as one group, so it carries at most the pass's rows
                const int per = std::max(1, (beam ? std::min(cap, e.max_rows()) : cap) / dchunk);
                for (size_t g0 = 0; g0 < grp.size(); g0 += per)
                for (int d0 = 0; d0 < ndec; d0 += dchunk) {
                    const int nj = (int)std::min<size_t>(per, grp.size() - g0);
                    const int nd = std::min(dchunk, ndec - d0);  // decoders d0 .. d0 + nd - 1
                    const int B = nj * nd;
                    DecodeRequest rq;
                    rq.prompt = prompt_init;
                    rq.full = true;
                    rq.flags = (p.suppress_blank ? 1u : 0u) | (p.no_timestamps ? 2u : 0u);
                    rq.ts.temperature = t_cur;
                    rq.ts.suppress_blank = p.suppress_blank ? 1 : 0;
                    rq.ts.no_ts = p.no_timestamps ? 1 : 0;
                    rq.ts.max_initial = max_initial;
                    rq.ts.n_max = n_max;
                    rq.ts.max_tokens = p.max_tokens;
                    rq.ts.seed = p.seed * 0x9E3779B97F4A7C15ULL + (++call);
                    rq.extra_suppress = nst;
                    rq.blank_tok = blank;
                    rq.n_steps = std::min(n_max, dm.n_text_ctx + 1 - P - Tq);
                    for (int j = 0; j < nj; ++j) {
                        const int u = grp[g0 + j];
                        for (int d = 0; d < nd; ++d) {
                            rq.kv_row.push_back(win_of.at(u));  // the utterance's encoded window
                            rq.seek.push_back(us[u].seek);
                            rq.seek_end.push_back(us[u].seek_end);
                            if (P > 0) rq.row_prefix.push_back(prefix[u]);
                            if (multi) rq.lang_tok.push_back(us[u].lang >= 0 ? us[u].lang : -(j * nd + 1));
                        }
                    }
                    if (no_share) {  // test hook: every row its own copy of its window (ABI <= 10)
                        std::vector<int> wu, ws;
                        for (int j = 0; j < nj; ++j)
                            for (int d = 0; d < nd; ++d) {
                                wu.push_back(chunk_utt.at(grp[g0 + j]));
                                ws.push_back(us[grp[g0 + j]].seek);
                            }
                        e.encode_windows(wu.data(), ws.data(), B);
                        rq.kv_row.clear();
                    }
                    if (beam) {
                        rq.beam_k = ndec;
                        std::vector<std::vector<DecOut>> bo;
                        std::vector<int> lang;
                        run_beam(e, rq, nj, nd, rq.seek, rq.seek_end, p, sp, n_max, &bo, &lang);
                        for (int j = 0; j < nj; ++j) {
                            const int u = grp[g0 + j];
                            if (multi && us[u].lang < 0) {
                                us[u].lang = lang[j * nd];
                                (*out)[u].lang_tok = us[u].lang;
                            }
                            res[u] = std::move(bo[j]);
                        }
                        continue;
                    }
                    const int S = rq.n_steps;
                    std::vector<int> tok((size_t)B * S), lang(B, -1), state((size_t)B * 4);
                    std::vector<float> plog((size_t)B * S), tid((size_t)B * S);
                    e.decode(B, rq, tok.data(), plog.data(), tid.data(), lang.data(), state.data());
                    for (int j = 0; j < nj; ++j) {
                        const int u = grp[g0 + j];
                        if (multi && us[u].lang < 0) {  // detected once, on the utterance's first window
                            us[u].lang = lang[j * nd];
                            (*out)[u].lang_tok = us[u].lang;
                        }
                        std::vector<DecOut>& ds = res[u];
                        for (int d = 0; d < nd; ++d) {
                            const int r = j * nd + d;
                            DecOut o;
                            for (int s = 0; s < S; ++s) {
                                const int tk = tok[(size_t)r * S + s];
                                if (tk < 0) break;
                                o.tok.push_back(tk);
                                o.plog.push_back(plog[(size_t)r * S + s]);
                                o.tid.push_back(tid[(size_t)r * S + s]);
                            }
                            o.seek_delta = state[r * 4 + 1];
                            o.result_len = state[r * 4 + 2];
                            o.status = state[r * 4 + 3];
                            o.failed = o.status == 2;
                            ds.push_back(std::move(o));
                        }
                    }
                }
            }
            std::vector<int> again;
            for (int u : pending) {
                std::vector<DecOut>& ds = res[u];
                int best = 0;
                double best_score = -INFINITY;
                for (int d = 0; d < (int)ds.size(); ++d) {
                    score(ds[d], p);
                    if (!ds[d].failed && best_score < ds[d].score) {
                        best_score = ds[d].score;
                        best = d;
                    }
                }
                const DecOut& bd = ds[best];
                if (it + 1 < temps.size() && (bd.failed || bd.avg < p.logprob_thold)) {
                    again.push_back(u);  // fall back to the next temperature
                    continue;
                }
                // the window's result (a failed decoder keeps every generated token)
                FullResult& r = (*out)[u];
                Utt& us_u = us[u];
                const int len = bd.failed ? (int)bd.tok.size() : std::min<int>(bd.result_len, (int)bd.tok.size());
                const int base = (int)r.tokens.size();
                r.tokens.insert(r.tokens.end(), bd.tok.begin(), bd.tok.begin() + len);
                r.plog.insert(r.plog.end(), bd.plog.begin(), bd.plog.begin() + len);
                r.tid.insert(r.tid.end(), bd.tid.begin(), bd.tid.begin() + len);
                r.n_windows++;
                r.n_fallbacks += (int)it;
                // prompt_past: the conditioning tokens just used (without [prev]) + the result
                const std::vector<int>& pf = prefix[u];
                std::vector<int> past;
                if (!pf.empty()) past.assign(pf.begin() + 1, pf.end());
                for (int i = 0; i < bd.result_len && i < (int)bd.tok.size(); ++i) past.push_back(bd.tok[i]);
                us_u.past.swap(past);
                // segments: split at timestamp tokens, text from the text tokens
                auto text_of = [&](int t) { return vocab ? vocab->str(t) : "[" + std::to_string(t) + "]"; };
                if (len > 0) {
                    int i0 = 0;
                    int64_t t0 = us_u.seek + 2 * ((int64_t)bd.tid[0] - sp.beg);
                    std::string text;
                    for (int i = 0; i < len; ++i) {
                        const int tk = bd.tok[i];
                        if (tk < sp.eot) text += text_of(tk);
                        if (tk > sp.beg) {
                            const int64_t t1 = us_u.seek + 2 * ((int64_t)bd.tid[i] - sp.beg);
                            if (!text.empty()) r.segments.push_back(FullSegment{t0, t1, text, base + i0, i - i0 + 1});
                            text.clear();
                            while (i < len && bd.tok[i] > sp.beg) ++i;
                            --i;
                            t0 = t1;
                            i0 = i + 1;
                        }
                    }
                    if (!text.empty())
                        r.segments.push_back(FullSegment{t0, us_u.seek + bd.seek_delta, text, base + i0, len - i0});
                }
                // a decoder that made no progress would repeat the window forever: skip it whole
                us_u.seek += bd.seek_delta > 0 ? bd.seek_delta : 3000;
            }
            pending.swap(again);
        }
    };
    // utterances in sets whose PCM and log-mel stay resident together (an hour of audio per set;
    // a longer utterance is a set of its own): each set's log-mel is computed once, whole
    constexpr int64_t kSetSamples = 16000LL * 3600;
    for (int u0 = 0; u0 < U;) {
        int u1 = u0;
        int64_t tot = 0;
        while (u1 < U && (u1 == u0 || tot + n[u1] <= kSetSamples)) tot += n[u1++];
        bool any = false;
        for (int u = u0; u < u1; ++u) any = any || us[u].seek + 100 < us[u].seek_end;
        if (any) e.load_utterances(pcm.data() + u0, n.data() + u0, u1 - u0);
        while (any) {
            std::vector<int> act;
            for (int u = u0; u < u1; ++u) {
                if (us[u].done) continue;
                if (us[u].seek + 100 >= us[u].seek_end) { us[u].done = true; continue; }  // < 1 s left
                act.push_back(u);
            }
            if (act.empty()) break;
            for (int u : act)  // a short tail: drop the past prompt (it makes the decoder repeat itself)
                if (us[u].seek > 0 && us[u].seek + 500 >= us[u].seek_end) us[u].past.clear();
            // one encoder run per window (whisper_encode_internal at `seek`), shared by every
            // temperature and every decoder of the utterance
            for (size_t c0 = 0; c0 < act.size(); c0 += cap) {
                const std::vector<int> chunk(act.begin() + c0, act.begin() + std::min(act.size(), c0 + cap));
                const int E = (int)chunk.size();
                std::vector<int> wu(E), ws(E);
                std::map<int, int> win_of;
                for (int i = 0; i < E; ++i) {
                    wu[i] = chunk[i] - u0;
                    chunk_utt[chunk[i]] = wu[i];
                    ws[i] = us[chunk[i]].seek;
                    win_of[chunk[i]] = i;
                }
                e.encode_windows(wu.data(), ws.data(), E);
                window_pass(chunk, win_of);
            }
        }
        u0 = u1;
    }
    for (FullResult& r : *out)
        for (const FullSegment& s : r.segments) r.text += s.text;
}

}  // namespace spt
