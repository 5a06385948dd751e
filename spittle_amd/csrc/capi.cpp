// capi.cpp -- the extern "C" boundary declared in include/spittle_hip.h.
//
// Mirrors transcribe-rs' WhisperEngine surface as Spittle uses it
// (/root/reference/src-tauri/src/managers/transcription.rs: new + load_model 261-276,
// transcribe_samples 494-503, unload_model 175-208): status codes + message,
// borrowed input PCM, library-owned results.  The fast path (no timestamps, greedy, no
// fallback) decodes one-window utterances; longer or sub-second ones take whisper_full's
// seek loop at the same parameters (spt_transcribe_batch).  Only the benchmark / test hooks
// (SPT_IGNORE_EOT, forced tokens) cut an utterance into fixed 30 s windows of its whole
// log-mel (frames 3000 k ..), independent batch items whose text is concatenated.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/spittle_hip.h"
#include "common.h"
#include "engine.h"
#include "full.h"
#include "ggml_file.h"
#include "vocab.h"

using spt::Engine;

#include "capi_internal.h"

namespace {

constexpr int kWindow = 480000;

void set_err(char* buf, size_t len, const std::string& msg) {
    if (buf && len) {
        strncpy(buf, msg.c_str(), len - 1);
        buf[len - 1] = 0;
    }
}

}  // namespace

spt_status spt_fail(spt_ctx* c, spt_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

spt_status spt_classify(const std::exception& e) {
    if (dynamic_cast<const spt::HipError*>(&e)) return SPT_ERR_DEVICE;
    if (dynamic_cast<const std::bad_alloc*>(&e)) return SPT_ERR_OOM;
    const std::string m = e.what();
    if (m.find("out of device memory") != std::string::npos) return SPT_ERR_OOM;
    return SPT_ERR_INVALID_ARG;
}

namespace {

spt_status fail(spt_ctx* c, spt_status s, const std::string& msg) { return spt_fail(c, s, msg); }
spt_status classify(const std::exception& e) { return spt_classify(e); }

// whisper_full: initial_prompt is tokenised (whisper_tokenize) only when no prompt_tokens are
// given; either way the tokens become the prompt_past
spt_status prompt_tokens_of(spt_ctx* c, const spt_infer_params* p, std::vector<int32_t>* out) {
    out->clear();
    if (p->prompt_tokens && p->n_prompt_tokens > 0) {
        out->assign(p->prompt_tokens, p->prompt_tokens + p->n_prompt_tokens);
    } else if (p->initial_prompt && p->initial_prompt[0]) {
        if (!c->vocab)
            return fail(c, SPT_ERR_UNSUPPORTED,
                        "initial_prompt text needs the tokenizer vocabulary of a ggml model; pass prompt_tokens");
        const std::vector<int> t = c->vocab->tokenize(p->initial_prompt, nullptr);
        out->assign(t.begin(), t.end());
    }
    for (int32_t t : *out)
        if (t < 0 || t >= c->eng->dims().n_vocab) return fail(c, SPT_ERR_INVALID_ARG, "prompt token out of the vocabulary");
    return SPT_OK;
}

// language of a request: >= 0 the fixed language token, -1 auto-detect, -2 English-only model
spt_status lang_of(spt_ctx* c, const spt_infer_params* p, int* lang_tok) {
    const spt::Specials sp = spt::specials_for(c->eng->dims().n_vocab);
    if (sp.n_langs <= 0) { *lang_tok = -2; return SPT_OK; }
    if (!p->language || !p->language[0] || std::string(p->language) == "auto") { *lang_tok = -1; return SPT_OK; }
    const int lid = spt::lang_id(p->language);
    if (lid < 0 || lid >= sp.n_langs) return fail(c, SPT_ERR_INVALID_ARG, std::string("unknown language '") + p->language + "'");
    *lang_tok = sp.sot + 1 + lid;
    return SPT_OK;
}

// the device-resident greedy no-timestamp protocol, or whisper_full's window loop
bool full_mode(const spt_infer_params* p) {
    return !(p->flags & SPT_NO_TIMESTAMPS) || p->temperature_inc > 0.0f || p->temperature != 0.0f || p->beam_size > 1;
}

// whisper_full's prompt_init: [sot] (+ [lang, task] for multilingual) + [notimestamps]; its
// prompt_past ([prev] + the last n_text_ctx / 2 prompt tokens) goes to rq->prefix.  With no
// language (the app's "auto", settings.rs:925) *auto is set and the caller fills rq->lang_tok.
spt_status build_request(spt_ctx* c, const spt_infer_params* p, spt::DecodeRequest* rq, bool* autolang) {
    spt_infer_params d;
    spt_default_infer_params(&d);
    if (!p) p = &d;
    const spt::ModelDims& dm = c->eng->dims();
    const spt::Specials sp = spt::specials_for(dm.n_vocab);
    *autolang = false;
    if (p->beam_size > 1) return fail(c, SPT_ERR_UNSUPPORTED, "beam search is not implemented (greedy only)");
    std::vector<int32_t> ptoks;
    spt_status st = prompt_tokens_of(c, p, &ptoks);
    if (st != SPT_OK) return st;
    rq->prompt.clear();
    rq->prefix.clear();
    rq->lang_tok.clear();
    if (!ptoks.empty()) {
        const int np = (int)ptoks.size();
        const int n_take = std::min(np, dm.n_text_ctx / 2);
        rq->prefix.push_back(sp.prev);
        for (int i = np - n_take; i < np; ++i) {
            const int t = ptoks[i];
            if (t < 0 || t >= dm.n_vocab) return fail(c, SPT_ERR_INVALID_ARG, "prompt token out of the vocabulary");
            rq->prefix.push_back(t);
        }
    }
    rq->prompt.push_back(sp.sot);
    if (sp.n_langs > 0) {
        const bool autod = !p->language || !p->language[0] || std::string(p->language) == "auto";
        int lid = 0;
        if (!autod) {
            lid = spt::lang_id(p->language);
            if (lid < 0 || lid >= sp.n_langs)
                return fail(c, SPT_ERR_INVALID_ARG, std::string("unknown language '") + p->language + "'");
        }
        *autolang = autod;
        rq->prompt.push_back(sp.sot + 1 + lid);  // replaced per sequence when auto-detecting
        rq->prompt.push_back(p->translate ? sp.translate : sp.transcribe);
    }
    rq->prompt.push_back(sp.not_);  // the fast path is the no-timestamp protocol
    int n = p->max_new_tokens > 0 ? p->max_new_tokens : 220;
    const int used = (int)(rq->prefix.size() + rq->prompt.size());
    if (used + n > dm.n_text_ctx + 1) n = dm.n_text_ctx + 1 - used;
    rq->n_steps = n;
    rq->flags = p->flags;
    rq->forced = p->forced_tokens;
    rq->n_forced = p->forced_tokens ? p->n_forced : 0;
    if (rq->n_forced < 0 || rq->n_forced > dm.n_text_ctx) return fail(c, SPT_ERR_INVALID_ARG, "n_forced out of range");
    return SPT_OK;
}

// whisper_full's segment text: the token strings of the text tokens (ids >= eot are skipped);
// a synthetic model has no vocabulary and shows the ids as "[id]"
void append_text(const spt_ctx* c, std::string* text, int t) {
    if (c->vocab) *text += c->vocab->str(t);
    else *text += "[" + std::to_string(t) + "]";
}

int lang_index(int lang_tok, const spt::Specials& sp) { return lang_tok > sp.sot ? lang_tok - sp.sot - 1 : -1; }

spt_result* make_result(int n_windows, int language, std::vector<int>* acc_tok, std::vector<float>* acc1,
                        std::vector<float>* acc2, std::string* text) {
    spt_result* r = (spt_result*)calloc(1, sizeof(spt_result));
    if (!r) return nullptr;
    const size_t n = acc_tok->size();
    r->n_tokens = (int32_t)n;
    r->n_windows = n_windows;
    r->language = language;
    r->tokens = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
    r->top1 = (float*)malloc(sizeof(float) * (n ? n : 1));
    r->top2 = (float*)malloc(sizeof(float) * (n ? n : 1));
    r->text = (char*)malloc(text->size() + 1);
    if (!r->tokens || !r->top1 || !r->top2 || !r->text) {
        spt_result_free(r);
        return nullptr;
    }
    for (size_t i = 0; i < n; ++i) {
        r->tokens[i] = (*acc_tok)[i];
        r->top1[i] = (*acc1)[i];
        r->top2[i] = (*acc2)[i];
    }
    memcpy(r->text, text->c_str(), text->size() + 1);
    return r;
}

// transcribe-rs joins the segment texts and trims the result (str::trim: ASCII whitespace here)
std::string trimmed(const std::string& s) {
    const char* ws = " \t\n\r\v\f";
    const size_t a = s.find_first_not_of(ws);
    if (a == std::string::npos) return std::string();
    return s.substr(a, s.find_last_not_of(ws) - a + 1);
}

spt_result* make_full_result(const spt::FullResult& f, const spt::Specials& sp) {
    std::vector<int> tok = f.tokens;
    std::vector<float> a = f.plog, b = f.tid;
    std::string text = trimmed(f.text);
    spt_result* r = make_result(f.n_windows, lang_index(f.lang_tok, sp), &tok, &a, &b, &text);
    if (!r) return nullptr;
    r->n_fallbacks = f.n_fallbacks;
    const size_t ns = f.segments.size();
    r->segments = (spt_segment*)calloc(ns ? ns : 1, sizeof(spt_segment));
    if (!r->segments) { spt_result_free(r); return nullptr; }
    r->n_segments = (int32_t)ns;
    for (size_t i = 0; i < ns; ++i) {
        const spt::FullSegment& s = f.segments[i];
        spt_segment& o = r->segments[i];
        o.t0 = s.t0; o.t1 = s.t1; o.i0 = s.i0; o.n_tokens = s.n;
        o.text = (char*)malloc(s.text.size() + 1);
        if (!o.text) { spt_result_free(r); return nullptr; }
        memcpy(o.text, s.text.c_str(), s.text.size() + 1);
    }
    return r;
}

// whisper_full (full.cpp) over host utterances
spt_status run_full(spt_ctx* c, const float* const* pcm, const size_t* n_samples, size_t batch,
                    const spt_infer_params* p, spt_result** out) {
    if (p->beam_size > 8) return fail(c, SPT_ERR_INVALID_ARG, "beam_size must be at most 8");
    if (p->beam_size > c->eng->max_batch())
        return fail(c, SPT_ERR_INVALID_ARG, "beam_size exceeds the context's max_batch (one row per beam)");
    if (p->forced_tokens || (p->flags & SPT_IGNORE_EOT))
        return fail(c, SPT_ERR_INVALID_ARG, "forced tokens / SPT_IGNORE_EOT are fast-path (no-timestamp) hooks");
    if ((p->flags & SPT_SUPPRESS_NST) && !c->vocab)
        return fail(c, SPT_ERR_UNSUPPORTED, "suppressing non-speech tokens needs the vocabulary of a ggml model");
    if (p->temperature < 0.0f || p->temperature_inc < 0.0f) return fail(c, SPT_ERR_INVALID_ARG, "negative temperature");
    std::vector<int32_t> ptoks;
    spt_status st = prompt_tokens_of(c, p, &ptoks);
    if (st != SPT_OK) return st;
    int lang_tok;
    st = lang_of(c, p, &lang_tok);
    if (st != SPT_OK) return st;
    spt::FullParams fp;
    fp.no_timestamps = (p->flags & SPT_NO_TIMESTAMPS) != 0;
    fp.suppress_blank = (p->flags & SPT_SUPPRESS_BLANK) != 0;
    fp.suppress_nst = (p->flags & SPT_SUPPRESS_NST) != 0;
    fp.translate = p->translate != 0;
    fp.temperature = p->temperature;
    fp.temperature_inc = p->temperature_inc;
    fp.best_of = p->best_of > 0 ? p->best_of : 5;
    fp.beam_size = std::max(1, p->beam_size);
    fp.entropy_thold = p->entropy_thold;
    fp.logprob_thold = p->logprob_thold;
    fp.max_initial_ts = p->max_initial_ts;
    fp.max_tokens = std::max(0, p->max_new_tokens);
    fp.seed = p->seed;
    std::vector<const float*> ptr(batch);
    std::vector<int> ns(batch);
    for (size_t u = 0; u < batch; ++u) {
        if (n_samples[u] > (size_t)INT32_MAX / 2) return fail(c, SPT_ERR_INVALID_ARG, "utterance too long");
        ptr[u] = pcm[u];
        ns[u] = (int)n_samples[u];
    }
    const spt::Specials sp = spt::specials_for(c->eng->dims().n_vocab);
    std::vector<spt::FullResult> res;
    spt::whisper_full_batch(*c->eng, c->vocab.get(), ptr, ns, fp, std::vector<int>(ptoks.begin(), ptoks.end()),
                            lang_tok >= 0 ? lang_tok : -1, &res);
    for (size_t u = 0; u < batch; ++u) {
        out[u] = make_full_result(res[u], sp);
        if (!out[u]) {
            for (size_t v = 0; v < u; ++v) { spt_result_free(out[v]); out[v] = nullptr; }
            return fail(c, SPT_ERR_OOM, "host allocation failed");
        }
    }
    return SPT_OK;
}

// shared driver: 30 s windows of host utterances -> per-utterance results.  Window k of an
// utterance starts at frame 3000 k of the utterance's whole log-mel (whisper_full with
// no_timestamps advances seek by 3000 frames per window).
struct Window { int utt; int seek; };

spt_status run_windows(spt_ctx* c, std::vector<Window>& win, const float* const* pcm, const size_t* n_samples,
                       size_t n_utt, const spt_infer_params* p, spt_result** out) {
    spt::DecodeRequest rq;
    bool autolang = false;
    spt_status s = build_request(c, p, &rq, &autolang);
    if (s != SPT_OK) return s;
    Engine& e = *c->eng;
    const spt::Specials sp = spt::specials_for(e.dims().n_vocab);
    const int eot = sp.eot;
    std::vector<std::vector<int>> tok(n_utt);
    std::vector<std::vector<float>> t1(n_utt), t2(n_utt);
    std::vector<std::string> text(n_utt);
    std::vector<int> nwin(n_utt, 0);
    // language per utterance: fixed, or detected on its first window (whisper_full detects once
    // per call from offset 0); later windows reuse it
    std::vector<int> utt_lang(n_utt, (!autolang && rq.prompt.size() >= 3) ? rq.prompt[1] : -1);
    const int cap = e.max_batch();
    std::vector<int> loaded;  // the utterances whose PCM and whole log-mel are resident
    for (size_t g0 = 0; g0 < win.size(); g0 += cap) {
        const int B = (int)std::min<size_t>(cap, win.size() - g0);
        // the utterances of this batch of windows, each log-mel computed whole.  An utterance whose
        // windows span several batches stays loaded while the batches hold only it (one long
        // recording: loaded once, not once per batch of windows -- ADVICE r4)
        std::vector<const float*> up;
        std::vector<int> un, uid, wu(B), ws(B);
        for (int b = 0; b < B; ++b) {
            const int u = win[g0 + b].utt;
            if (b == 0 || win[g0 + b - 1].utt != u) {
                up.push_back(pcm[u]);
                un.push_back((int)n_samples[u]);
                uid.push_back(u);
            }
            wu[b] = (int)up.size() - 1;
            ws[b] = win[g0 + b].seek;
        }
        if (autolang) {
            rq.lang_tok.assign(B, 0);
            for (int b = 0; b < B; ++b) {
                const int u = win[g0 + b].utt;
                if (utt_lang[u] >= 0) { rq.lang_tok[b] = utt_lang[u]; continue; }
                int src = b;  // the utterance's first window in this batch
                while (src > 0 && win[g0 + src - 1].utt == u) --src;
                rq.lang_tok[b] = -(src + 1);
            }
        }
        std::vector<int> otok((size_t)B * rq.n_steps), lang(B, -1);
        std::vector<float> o1((size_t)B * rq.n_steps), o2((size_t)B * rq.n_steps);
        if (uid != loaded) {
            e.load_utterances(up.data(), un.data(), (int)up.size());
            loaded = uid;
        }
        e.encode_windows(wu.data(), ws.data(), B);
        e.decode(B, rq, otok.data(), o1.data(), o2.data(), lang.data());
        for (int b = 0; b < B; ++b) {
            const int u = win[g0 + b].utt;
            if (utt_lang[u] < 0) utt_lang[u] = lang[b];
            nwin[u]++;
            for (int s2 = 0; s2 < rq.n_steps; ++s2) {
                const int t = otok[(size_t)b * rq.n_steps + s2];
                if (t < 0) break;
                tok[u].push_back(t);
                t1[u].push_back(o1[(size_t)b * rq.n_steps + s2]);
                t2[u].push_back(o2[(size_t)b * rq.n_steps + s2]);
                if (t < eot) append_text(c, &text[u], t);
                if (t == eot && !(rq.flags & SPT_IGNORE_EOT)) break;
            }
        }
    }
    for (size_t u = 0; u < n_utt; ++u) {
        out[u] = make_result(nwin[u], lang_index(utt_lang[u], sp), &tok[u], &t1[u], &t2[u], &text[u]);
        if (!out[u]) {
            for (size_t v = 0; v < u; ++v) { spt_result_free(out[v]); out[v] = nullptr; }
            return fail(c, SPT_ERR_OOM, "host allocation failed");
        }
    }
    return SPT_OK;
}

}  // namespace

extern "C" {

const char* spt_version(void) { return "spittle_amd 0.12.0 (gfx950, ABI 12)"; }

const char* spt_language_code(int32_t lang_id) { return spt::lang_code(lang_id); }

void spt_default_model_params(spt_model_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->dtype = SPT_DTYPE_BF16;
    p->device = 0;
    p->max_batch = 8;
    p->seed = 1234;
}

void spt_default_infer_params(spt_infer_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->language = "en";
    p->flags = SPT_SUPPRESS_BLANK;  // whisper_full_default_params: timestamps on
    p->max_new_tokens = 220;
    p->temperature = 0.0f;
    p->beam_size = 1;
    p->temperature_inc = 0.2f;
    p->best_of = 5;
    p->entropy_thold = 2.4f;
    p->logprob_thold = -1.0f;
    p->max_initial_ts = 1.0f;
}

spt_status spt_ctx_create(const char* model_spec, const spt_model_params* params, spt_ctx** out, char* err,
                          size_t errlen) {
    if (!model_spec || !out) {
        set_err(err, errlen, "null argument");
        return SPT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    spt_model_params mp;
    spt_default_model_params(&mp);
    if (params) mp = *params;
    if (mp.dtype != SPT_DTYPE_F32 && mp.dtype != SPT_DTYPE_BF16) {
        set_err(err, errlen, "bad dtype");
        return SPT_ERR_INVALID_ARG;
    }
    if (mp.flags & ~SPT_MODEL_WEIGHTS_EXTERNAL) {
        set_err(err, errlen, "unknown spt_model_params.flags bits");
        return SPT_ERR_INVALID_ARG;
    }
    spt::ModelDims dm;
    uint64_t seed = mp.seed;
    std::string perr;
    const std::string spec(model_spec);
    std::unique_ptr<spt::GgmlFile> file;
    if (!spt::parse_synthetic_spec(spec, &dm, &seed, &perr)) {
        FILE* f = fopen(model_spec, "rb");
        if (!f) {
            set_err(err, errlen, "model file not found: " + spec);
            return SPT_ERR_LOAD;
        }
        fclose(f);
        file.reset(new spt::GgmlFile());
        if (!file->open(spec, &perr) || !spt::ggml_dims(*file, &dm, &perr)) {
            set_err(err, errlen, spec + ": " + perr);
            return SPT_ERR_LOAD;
        }
        perr.clear();
    }
    if (!perr.empty()) {
        set_err(err, errlen, perr);
        return SPT_ERR_LOAD;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_err(err, errlen, "no HIP device available");
        return SPT_ERR_DEVICE;
    }
    if (mp.device < 0 || mp.device >= ndev) {
        set_err(err, errlen, "device ordinal out of range");
        return SPT_ERR_INVALID_ARG;
    }
    spt_ctx* c = new (std::nothrow) spt_ctx();
    if (!c) return SPT_ERR_OOM;
    try {
        c->eng.reset(new Engine(dm, mp.dtype == SPT_DTYPE_BF16 ? spt::DT_BF16 : spt::DT_F32, mp.device,
                                mp.max_batch, seed, file.get(), (mp.flags & SPT_MODEL_WEIGHTS_EXTERNAL) != 0));
        if (file) c->vocab.reset(new spt::Vocab(file->vocab(), dm.n_vocab, spt::specials_for(dm.n_vocab)));
    } catch (const std::exception& e) {
        set_err(err, errlen, e.what());
        const spt_status s = classify(e);
        delete c;
        return s == SPT_ERR_INVALID_ARG ? SPT_ERR_LOAD : s;
    }
    c->spec = spec;
    *out = c;
    return SPT_OK;
}

void spt_ctx_destroy(spt_ctx* ctx) { delete ctx; }

const char* spt_last_error(const spt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

spt_status spt_ctx_info(const spt_ctx* ctx, spt_model_info* info) {
    if (!ctx || !info) return SPT_ERR_INVALID_ARG;
    const spt::ModelDims& d = ctx->eng->dims();
    info->n_mels = d.n_mels; info->d = d.d; info->n_head = d.n_head; info->n_enc = d.n_enc; info->n_dec = d.n_dec;
    info->n_vocab = d.n_vocab; info->n_audio_ctx = d.n_audio_ctx; info->n_text_ctx = d.n_text_ctx;
    info->dtype = ctx->eng->dtype() == spt::DT_BF16 ? SPT_DTYPE_BF16 : SPT_DTYPE_F32;
    info->max_batch = ctx->eng->max_batch();
    info->weight_bytes = ctx->eng->weight_bytes();
    info->workspace_bytes = ctx->eng->workspace_bytes();
    return SPT_OK;
}

spt_status spt_transcribe_batch(spt_ctx* ctx, const float* const* pcm, const size_t* n_samples, size_t batch,
                                const spt_infer_params* params, spt_result** out) {
    if (!ctx || !out || (batch && (!pcm || !n_samples))) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    spt_infer_params dflt;
    spt_default_infer_params(&dflt);
    if (!params) params = &dflt;
    ctx->eng->reset_call_stats();
    if (full_mode(params)) {
        for (size_t u = 0; u < batch; ++u) {
            out[u] = nullptr;
            if (n_samples[u] && !pcm[u]) return fail(ctx, SPT_ERR_INVALID_ARG, "null pcm");
        }
        try {
            return batch ? run_full(ctx, pcm, n_samples, batch, params, out) : SPT_OK;
        } catch (const std::exception& e) {
            return fail(ctx, classify(e), e.what());
        }
    }
    // The fast path decodes one window at seek 0, which is exactly whisper_full's result for an input
    // of one window that passes its one-second check.  Other inputs take whisper_full's seek loop
    // (full.cpp, at these same parameters: no timestamps, greedy, no fallback), so they follow its
    // window rules: nothing under the one-second threshold (n_len_org < 100 frames), a window only
    // while seek + 100 < seek_end (480 001 samples decode one window, not two), and each later window
    // conditioned on the earlier windows' tokens (prompt_past).  The benchmark / test hooks
    // (SPT_IGNORE_EOT, forced tokens) have no whisper_full meaning and keep fixed 30 s windows.
    const bool hooks = (params->flags & SPT_IGNORE_EOT) || (params->forced_tokens && params->n_forced > 0);
    std::vector<Window> win;
    std::vector<size_t> empty, seek_loop;
    for (size_t u = 0; u < batch; ++u) {
        out[u] = nullptr;
        if (n_samples[u] == 0) { empty.push_back(u); continue; }  // "" without an engine call
        if (!pcm[u]) return fail(ctx, SPT_ERR_INVALID_ARG, "null pcm");
        if (n_samples[u] > (size_t)INT32_MAX / 2) return fail(ctx, SPT_ERR_INVALID_ARG, "utterance too long");
        const int n_len = 1 + ((int)n_samples[u] - 200) / 160;  // log_mel_spectrogram's n_len_org
        if (!hooks && (n_len < 100 || n_samples[u] > (size_t)kWindow)) { seek_loop.push_back(u); continue; }
        for (size_t o = 0; o < n_samples[u]; o += kWindow) win.push_back(Window{(int)u, (int)(o / 160)});
    }
    try {
        spt_status s = SPT_OK;
        if (!win.empty()) {
            // results for non-empty utterances
            std::vector<spt_result*> tmp(batch, nullptr);
            s = run_windows(ctx, win, pcm, n_samples, batch, params, tmp.data());
            if (s != SPT_OK) return s;
            for (size_t u = 0; u < batch; ++u) out[u] = tmp[u];
        }
        if (!seek_loop.empty()) {
            std::vector<const float*> sp;
            std::vector<size_t> sn;
            for (size_t u : seek_loop) { sp.push_back(pcm[u]); sn.push_back(n_samples[u]); }
            std::vector<spt_result*> tmp(seek_loop.size(), nullptr);
            s = run_full(ctx, sp.data(), sn.data(), sp.size(), params, tmp.data());
            if (s != SPT_OK) {
                for (size_t u = 0; u < batch; ++u) { spt_result_free(out[u]); out[u] = nullptr; }
                return s;
            }
            for (size_t i = 0; i < seek_loop.size(); ++i) out[seek_loop[i]] = tmp[i];
        }
        for (size_t u : empty) {
            if (out[u]) spt_result_free(out[u]);
            std::vector<int> t; std::vector<float> a, b; std::string txt;
            out[u] = make_result(0, -1, &t, &a, &b, &txt);
        }
        return SPT_OK;
    } catch (const std::exception& e) {
        // run_full may throw after run_windows filled out[]: no partial results with a failure status
        for (size_t u = 0; u < batch; ++u) { spt_result_free(out[u]); out[u] = nullptr; }
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_transcribe(spt_ctx* ctx, const float* pcm16k, size_t n_samples, const spt_infer_params* params,
                          spt_result** out) {
    if (!ctx || !out) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n_samples && !pcm16k) return fail(ctx, SPT_ERR_INVALID_ARG, "null pcm");
    const float* p = pcm16k;
    return spt_transcribe_batch(ctx, &p, &n_samples, 1, params, out);
}

spt_status spt_transcribe_batch_device(spt_ctx* ctx, const float* pcm_dev, size_t stride, const size_t* n_samples,
                                       size_t batch, const spt_infer_params* params, spt_result** out) {
    if (!ctx || !out || !pcm_dev || !n_samples || batch == 0) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (batch > (size_t)ctx->eng->max_batch()) return fail(ctx, SPT_ERR_INVALID_ARG, "batch exceeds max_batch");
    if (stride < (size_t)kWindow) return fail(ctx, SPT_ERR_INVALID_ARG, "device stride must be >= 480000");
    spt_infer_params dflt;
    spt_default_infer_params(&dflt);
    if (!params) params = &dflt;  // the defaults are whisper_full's (timestamps on): unsupported here
    ctx->eng->reset_call_stats();
    if (full_mode(params))
        return fail(ctx, SPT_ERR_UNSUPPORTED,
                    "device windows take the no-timestamp greedy protocol (SPT_NO_TIMESTAMPS, temperature_inc 0)");
    spt::DecodeRequest rq;
    bool autolang = false;
    spt_status s = build_request(ctx, params, &rq, &autolang);
    if (s != SPT_OK) return s;
    try {
        std::vector<int> ns(batch);
        if (autolang) {  // each window is its own utterance here
            rq.lang_tok.resize(batch);
            for (size_t b = 0; b < batch; ++b) rq.lang_tok[b] = -(int)(b + 1);
        }
        for (size_t b = 0; b < batch; ++b) {
            if (n_samples[b] > (size_t)kWindow) return fail(ctx, SPT_ERR_INVALID_ARG, "device windows hold <= 480000 samples");
            ns[b] = (int)n_samples[b];
        }
        Engine& e = *ctx->eng;
        const int B = (int)batch;
        std::vector<int> otok((size_t)B * rq.n_steps), lang(B, -1);
        std::vector<float> o1((size_t)B * rq.n_steps), o2((size_t)B * rq.n_steps);
        e.transcribe_device(pcm_dev, (int64_t)stride, ns.data(), B, rq, otok.data(), o1.data(), o2.data(), lang.data());
        const spt::Specials sp = spt::specials_for(e.dims().n_vocab);
        const int eot = sp.eot;
        for (int b = 0; b < B; ++b) {
            std::vector<int> t; std::vector<float> a, c2; std::string txt;
            for (int s2 = 0; s2 < rq.n_steps; ++s2) {
                const int tk = otok[(size_t)b * rq.n_steps + s2];
                if (tk < 0) break;
                t.push_back(tk);
                a.push_back(o1[(size_t)b * rq.n_steps + s2]);
                c2.push_back(o2[(size_t)b * rq.n_steps + s2]);
                if (tk < eot) append_text(ctx, &txt, tk);
                if (tk == eot && !(rq.flags & SPT_IGNORE_EOT)) break;
            }
            out[b] = make_result(1, lang_index(lang[b], sp), &t, &a, &c2, &txt);
        }
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

void spt_result_free(spt_result* r) {
    if (!r) return;
    for (int32_t i = 0; i < r->n_segments && r->segments; ++i) free(r->segments[i].text);
    free(r->segments);
    free(r->text);
    free(r->tokens);
    free(r->top1);
    free(r->top2);
    free(r);
}

spt_status spt_tokenize(spt_ctx* ctx, const char* text, int32_t* tokens, int32_t n_max, int32_t* n_out) {
    if (!ctx || !text || !n_out || (n_max > 0 && !tokens)) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (!ctx->vocab) return fail(ctx, SPT_ERR_UNSUPPORTED, "synthetic models have no vocabulary");
    try {
        const std::vector<int> t = ctx->vocab->tokenize(text, nullptr);
        *n_out = (int32_t)t.size();
        if ((int64_t)t.size() > n_max) return fail(ctx, SPT_ERR_INVALID_ARG, "token buffer too small");
        for (size_t i = 0; i < t.size(); ++i) tokens[i] = t[i];
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

const char* spt_token_to_str(const spt_ctx* ctx, int32_t id) {
    if (!ctx || !ctx->vocab || id < 0 || id >= ctx->vocab->size()) return nullptr;
    return ctx->vocab->str(id).c_str();
}

spt_status spt_get_timings(const spt_ctx* ctx, spt_timings* t) {
    if (!ctx || !t) return SPT_ERR_INVALID_ARG;
    const spt::Timings& m = ctx->eng->timings();
    t->mel_ms = m.mel_ms; t->encoder_ms = m.encoder_ms; t->cross_kv_ms = m.cross_kv_ms; t->decode_ms = m.decode_ms;
    t->total_ms = m.total_ms; t->h2d_ms = m.h2d_ms; t->n_decode_passes = m.n_decode_passes; t->batch = m.batch;
    return SPT_OK;
}

spt_status spt_get_call_stats(const spt_ctx* ctx, spt_call_stats* s) {
    if (!ctx || !s) return SPT_ERR_INVALID_ARG;
    const spt::CallStats& c = ctx->eng->call_stats();
    s->engine_calls = c.engine_calls; s->decoder_passes = c.decoder_passes; s->beam_steps = c.beam_steps;
    s->encoder_windows = c.encoder_windows;
    s->device_ms = c.device_ms; s->encoder_ms = c.encoder_ms; s->decode_ms = c.decode_ms;
    s->pd_passes = c.pd_passes; s->pd_fallbacks = c.pd_fallbacks;
    return SPT_OK;
}

spt_status spt_weights_export(spt_ctx* ctx, void* dev_dst, size_t bytes) {
    if (!ctx || !dev_dst) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        ctx->eng->export_weights(dev_dst, (int64_t)bytes);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_weights_import(spt_ctx* ctx, const void* dev_src, size_t bytes) {
    if (!ctx || !dev_src) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        ctx->eng->import_weights(dev_src, (int64_t)bytes);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_debug_mel(spt_ctx* ctx, const float* pcm16k, size_t n_samples, float* out) {
    if (!ctx || !out || (n_samples && !pcm16k)) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n_samples > (size_t)kWindow) return fail(ctx, SPT_ERR_INVALID_ARG, "window longer than 30 s");
    return spt_debug_mel_at(ctx, pcm16k, n_samples, 0, out);
}

spt_status spt_debug_mel_at(spt_ctx* ctx, const float* pcm16k, size_t n_samples, int32_t seek, float* out) {
    if (!ctx || !out || (n_samples && !pcm16k)) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n_samples > (size_t)INT32_MAX / 2) return fail(ctx, SPT_ERR_INVALID_ARG, "utterance too long");
    try {
        ctx->eng->debug_mel(pcm16k, (int)n_samples, seek, out);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_debug_encode(spt_ctx* ctx, const float* mel, float* out) {
    if (!ctx || !mel || !out) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        ctx->eng->debug_encode(mel, out);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_debug_weight_checksum(spt_ctx* ctx, int32_t tensor_id, double* out2) {
    if (!ctx || !out2) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        if (!ctx->eng->debug_weight_checksum(tensor_id, out2)) return fail(ctx, SPT_ERR_INVALID_ARG, "unknown tensor id");
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_debug_ggml_tokenize(const char* model_path, const char* text, int32_t* tokens, int32_t n_max,
                                   int32_t* n_out) {
    if (!model_path || !text || !n_out || (n_max > 0 && !tokens)) return SPT_ERR_INVALID_ARG;
    spt::GgmlFile f;
    std::string err;
    if (!f.open(model_path, &err)) return SPT_ERR_LOAD;
    spt::Vocab v(f.vocab(), f.hparams().n_vocab, spt::specials_for(f.hparams().n_vocab));
    const std::vector<int> t = v.tokenize(text, nullptr);
    *n_out = (int32_t)t.size();
    if ((int64_t)t.size() > n_max) return SPT_ERR_INVALID_ARG;
    for (size_t i = 0; i < t.size(); ++i) tokens[i] = t[i];
    return SPT_OK;
}

spt_status spt_debug_ggml_dequant(int32_t ggml_type, const void* src, int64_t n, float* dst) {
    if (!src || !dst || n < 0) return SPT_ERR_INVALID_ARG;
    int blck, bytes;
    spt::GgmlFile::type_block(ggml_type, &blck, &bytes);
    if (!blck) return SPT_ERR_UNSUPPORTED;
    if (n % blck) return SPT_ERR_INVALID_ARG;
    return spt::ggml_dequant_host(ggml_type, (const uint8_t*)src, n, dst) ? SPT_OK : SPT_ERR_UNSUPPORTED;
}

}  // extern "C"

extern "C" spt_status spt_probe_kernel(spt_ctx* ctx, int32_t kind, int32_t iters, double* avg_us, double* work,
                                       int32_t* work_is_flops) {
    if (!ctx || !avg_us || !work || !work_is_flops) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        int f = 0;
        *avg_us = ctx->eng->probe(kind, iters, work, &f);
        *work_is_flops = f;
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}
