// capi_pk.cpp -- the spt_parakeet_* half of include/spittle_hip.h (ABI 6).
//
// Mirrors transcribe-rs' ParakeetEngine as Spittle drives it (/root/reference/src-tauri/src/
// managers/transcription.rs: load_model_with_params 278-297, transcribe_samples with
// TimestampGranularity::Segment 505-513, unload 175-208): status codes + message, borrowed PCM,
// library-owned results.  Like the reference engine, a recording is decoded whole in one pass:
// an utterance longer than the context's max_seconds grows the workspace to its length (up to 20
// minutes and kMaxGrowBytes of workspace); only past that limit, or when the device has no room,
// is it cut into chunks on 80 ms (encoder frame) boundaries, batched and concatenated.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/spittle_hip.h"
#include "common.h"
#include "kernels.h"
#include "parakeet.h"
#include "pk_onnx.h"

namespace {
constexpr int64_t kMaxGrowBytes = 96ll << 30;  // workspace a long recording may grow to (of 288 GB HBM)
}

struct spt_pk_ctx {
    std::unique_ptr<spt::ParakeetEngine> eng;
    std::vector<std::string> pieces;
    std::string spec, err;
};

struct spt_pk_onnx {  // a parsed model directory (host memory only)
    spt::PkOnnxModel m;
};

namespace {

constexpr int kFrameSamples = 1280;  // one encoder frame: 8 x 160 samples
constexpr double kFrameSec = 0.08;

spt_status fail(spt_pk_ctx* c, spt_status s, const std::string& m) {
    if (c) c->err = m;
    return s;
}

spt_status classify(const std::exception& e) {
    if (dynamic_cast<const spt::HipError*>(&e)) return SPT_ERR_DEVICE;
    if (dynamic_cast<const std::bad_alloc*>(&e)) return SPT_ERR_OOM;
    if (std::string(e.what()).find("out of device memory") != std::string::npos) return SPT_ERR_OOM;
    return SPT_ERR_INVALID_ARG;
}

void set_err(char* buf, size_t len, const std::string& m) {
    if (buf && len) {
        strncpy(buf, m.c_str(), len - 1);
        buf[len - 1] = 0;
    }
}

const char kWordMark[] = "\xE2\x96\x81";  // U+2581, SentencePiece's word-start marker

std::string piece_of(const spt_pk_ctx* c, int t) {
    if (t >= 0 && (size_t)t < c->pieces.size()) return c->pieces[t];
    return "[" + std::to_string(t) + "]";
}

std::string detok(const std::string& s) {
    std::string o;
    for (size_t i = 0; i < s.size();) {
        if (s.compare(i, 3, kWordMark) == 0) { o += ' '; i += 3; }
        else o += s[i++];
    }
    return o;
}

std::string trim(const std::string& s) {
    const char* ws = " \t\n\r\v\f";
    const size_t a = s.find_first_not_of(ws);
    if (a == std::string::npos) return std::string();
    return s.substr(a, s.find_last_not_of(ws) - a + 1);
}

struct Unit { int i0, n; };

// timestamp units of a token sequence: tokens, words (a piece starting with the word marker opens
// a word; without a vocabulary every token is one), or sentence segments (a word ending in . ? !
// closes one; without a vocabulary the whole utterance is one) [transcribe-rs, recalled]
std::vector<Unit> units_of(const spt_pk_ctx* c, const std::vector<int>& tok, int gran) {
    std::vector<Unit> u;
    const int n = (int)tok.size();
    if (!n) return u;
    const bool voc = !c->pieces.empty();
    if (gran == SPT_PK_TS_TOKEN || (!voc && gran == SPT_PK_TS_WORD)) {
        for (int i = 0; i < n; ++i) u.push_back(Unit{i, 1});
        return u;
    }
    std::vector<Unit> words;
    for (int i = 0; i < n; ++i) {
        const std::string p = piece_of(c, tok[i]);
        if (words.empty() || (voc && p.compare(0, 3, kWordMark) == 0)) words.push_back(Unit{i, 1});
        else words.back().n++;
    }
    if (gran == SPT_PK_TS_WORD) return words;
    if (!voc) return std::vector<Unit>{Unit{0, n}};
    Unit cur{words[0].i0, 0};
    for (const Unit& w : words) {
        cur.n = w.i0 + w.n - cur.i0;
        const std::string last = trim(detok(piece_of(c, tok[w.i0 + w.n - 1])));
        const char e = last.empty() ? 0 : last.back();
        if (e == '.' || e == '?' || e == '!') {
            u.push_back(cur);
            cur = Unit{w.i0 + w.n, 0};
        }
    }
    if (cur.n > 0) u.push_back(cur);
    return u;
}

spt_pk_result* make_result(const spt_pk_ctx* c, const spt::PkUtt& r, int n_chunks, int gran) {
    spt_pk_result* o = (spt_pk_result*)calloc(1, sizeof(spt_pk_result));
    if (!o) return nullptr;
    const size_t n = r.tok.size();
    o->n_tokens = (int32_t)n;
    o->n_chunks = n_chunks;
    o->tokens = (int32_t*)malloc(4 * (n ? n : 1));
    o->frames = (int32_t*)malloc(4 * (n ? n : 1));
    o->logit = (float*)malloc(4 * (n ? n : 1));
    o->runner_up = (float*)malloc(4 * (n ? n : 1));
    std::string text;
    for (size_t i = 0; i < n; ++i) text += piece_of(c, r.tok[i]);
    text = trim(detok(text));
    o->text = (char*)malloc(text.size() + 1);
    const std::vector<Unit> units = units_of(c, r.tok, gran);
    o->segments = (spt_pk_segment*)calloc(units.size() ? units.size() : 1, sizeof(spt_pk_segment));
    if (!o->tokens || !o->frames || !o->logit || !o->runner_up || !o->text || !o->segments) {
        spt_parakeet_result_free(o);
        return nullptr;
    }
    for (size_t i = 0; i < n; ++i) {
        o->tokens[i] = r.tok[i];
        o->frames[i] = r.frame[i];
        o->logit[i] = r.top1[i];
        o->runner_up[i] = r.top2[i];
    }
    memcpy(o->text, text.c_str(), text.size() + 1);
    o->n_segments = (int32_t)units.size();
    for (size_t k = 0; k < units.size(); ++k) {
        const Unit& u = units[k];
        spt_pk_segment& s = o->segments[k];
        s.i0 = u.i0;
        s.n_tokens = u.n;
        s.start = r.frame[u.i0] * kFrameSec;
        s.end = (r.frame[u.i0 + u.n - 1] + 1) * kFrameSec;
        std::string t;
        for (int i = 0; i < u.n; ++i) t += piece_of(c, r.tok[u.i0 + i]);
        t = trim(detok(t));
        s.text = (char*)malloc(t.size() + 1);
        if (!s.text) {
            spt_parakeet_result_free(o);
            return nullptr;
        }
        memcpy(s.text, t.c_str(), t.size() + 1);
    }
    return o;
}

spt_status check_params(spt_pk_ctx* c, const spt_pk_infer_params* p) {
    if (p->max_symbols < 1 || p->max_symbols > 16) return fail(c, SPT_ERR_INVALID_ARG, "max_symbols must be in [1, 16]");
    if (p->timestamp_granularity < SPT_PK_TS_TOKEN || p->timestamp_granularity > SPT_PK_TS_SEGMENT)
        return fail(c, SPT_ERR_INVALID_ARG, "bad timestamp_granularity");
    return SPT_OK;
}

}  // namespace

extern "C" {

void spt_parakeet_default_model_params(spt_pk_model_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->dtype = SPT_DTYPE_F16;
    p->max_batch = 8;
    p->max_seconds = 30.0f;
    p->seed = 1234;
}

void spt_parakeet_default_infer_params(spt_pk_infer_params* p) {
    if (!p) return;
    p->max_symbols = 10;  // NeMo's TDT greedy default
    p->timestamp_granularity = SPT_PK_TS_SEGMENT;  // what the app asks for (transcription.rs:505-513)
}

spt_status spt_parakeet_create(const char* model_spec, const spt_pk_model_params* params, spt_pk_ctx** out, char* err,
                               size_t errlen) {
    if (!model_spec || !out) {
        set_err(err, errlen, "null argument");
        return SPT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    spt_pk_model_params mp;
    spt_parakeet_default_model_params(&mp);
    if (params) mp = *params;
    if (mp.dtype != SPT_DTYPE_F32 && mp.dtype != SPT_DTYPE_F16 && mp.dtype != SPT_DTYPE_BF16) {
        set_err(err, errlen, "bad dtype");
        return SPT_ERR_INVALID_ARG;
    }
    if (mp.flags & ~SPT_PK_WEIGHTS_EMPTY) {
        set_err(err, errlen, "unknown spt_pk_model_params.flags bits");
        return SPT_ERR_INVALID_ARG;
    }
    if (!(mp.max_seconds >= 0.08f && mp.max_seconds <= 1200.0f)) {
        set_err(err, errlen, "max_seconds must be in [0.08, 1200]");
        return SPT_ERR_INVALID_ARG;
    }
    if (mp.max_batch < 1 || mp.max_batch > 64) {
        set_err(err, errlen, "max_batch must be in [1, 64]");
        return SPT_ERR_INVALID_ARG;
    }
    spt::PkDims dm;
    uint64_t seed = mp.seed;
    std::string perr;
    // the app's model directory (catalog parakeet-tdt-0.6b-v3-int8: the onnx-asr export), parsed on
    // the host before any device work; or a synthetic spec
    std::unique_ptr<spt::PkOnnxModel> onnx;
    if (spt::is_parakeet_onnx_dir(model_spec)) {
        onnx.reset(new (std::nothrow) spt::PkOnnxModel());
        if (!onnx) return SPT_ERR_OOM;
        try {
            if (!spt::load_parakeet_onnx(model_spec, onnx.get(), &perr)) {
                set_err(err, errlen, perr);
                return SPT_ERR_LOAD;
            }
        } catch (const std::exception& e) {  // std::bad_alloc on absurd shapes
            set_err(err, errlen, std::string("loading ") + model_spec + ": " + e.what());
            return SPT_ERR_LOAD;
        }
        dm = onnx->dims;
        mp.flags |= SPT_PK_WEIGHTS_EMPTY;
    } else if (!spt::parse_parakeet_spec(model_spec, &dm, &seed, &perr)) {
        set_err(err, errlen, std::string("unsupported Parakeet model '") + model_spec +
                                 "': expected the model directory (encoder-model[.int8].onnx, decoder_joint-model[.int8].onnx, "
                                 "vocab.txt) or a synthetic spec");
        return SPT_ERR_LOAD;
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
    // chunks end on encoder-frame boundaries
    const int max_samples = std::max(kFrameSamples, (int)(mp.max_seconds * 16000.0f) / kFrameSamples * kFrameSamples);
    spt_pk_ctx* c = new (std::nothrow) spt_pk_ctx();
    if (!c) return SPT_ERR_OOM;
    try {
        const int dt = mp.dtype == SPT_DTYPE_F16 ? spt::DT_F16 : mp.dtype == SPT_DTYPE_BF16 ? spt::DT_BF16 : spt::DT_F32;
        c->eng.reset(new spt::ParakeetEngine(dm, dt, mp.device, mp.max_batch, max_samples, seed,
                                             !(mp.flags & SPT_PK_WEIGHTS_EMPTY)));
        if (onnx) {
            for (int tid : c->eng->tensor_ids())
                if (!onnx->tensors.count(tid))
                    throw std::runtime_error(std::string(model_spec) + ": no tensor for " + spt::pk_tensor_name(tid));
            for (auto& kv : onnx->tensors) {  // host copies freed as they land
                c->eng->set_tensor(kv.first, kv.second.data(), (int64_t)kv.second.size());
                std::vector<float>().swap(kv.second);
            }
            c->pieces = onnx->pieces;
        }
    } catch (const std::exception& e) {
        set_err(err, errlen, e.what());
        const spt_status s = classify(e);
        delete c;
        return s == SPT_ERR_INVALID_ARG ? SPT_ERR_LOAD : s;
    }
    c->spec = model_spec;
    *out = c;
    return SPT_OK;
}

void spt_parakeet_destroy(spt_pk_ctx* ctx) { delete ctx; }

spt_status spt_parakeet_onnx_open(const char* dir, spt_pk_onnx** out, spt_pk_model_info* info, char* err,
                                  size_t errlen) {
    if (!dir || !out) {
        set_err(err, errlen, "null argument");
        return SPT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    if (!spt::is_parakeet_onnx_dir(dir)) {
        set_err(err, errlen, std::string(dir) + ": not a Parakeet model directory (no encoder-model[.int8].onnx)");
        return SPT_ERR_LOAD;
    }
    std::unique_ptr<spt_pk_onnx> h(new (std::nothrow) spt_pk_onnx());
    if (!h) return SPT_ERR_OOM;
    std::string e;
    try {
        if (!spt::load_parakeet_onnx(dir, &h->m, &e)) {
            set_err(err, errlen, e);
            return SPT_ERR_LOAD;
        }
    } catch (const std::exception& x) {
        set_err(err, errlen, std::string("loading ") + dir + ": " + x.what());
        return SPT_ERR_LOAD;
    }
    if (info) {
        memset(info, 0, sizeof(*info));
        const spt::PkDims& d = h->m.dims;
        info->n_mels = d.n_mels; info->d = d.d; info->n_layers = d.n_layers; info->n_heads = d.n_heads; info->ff = d.ff;
        info->sub_ch = d.sub_ch; info->conv_k = d.conv_k; info->pred = d.pred; info->n_vocab = d.n_vocab;
        info->n_dur = d.n_dur;
        info->reserved0 = h->m.n_quantized;
    }
    *out = h.release();
    return SPT_OK;
}

int64_t spt_parakeet_onnx_tensor(const spt_pk_onnx* h, int32_t tensor_id, const float** data) {
    if (!h || !data) return -1;
    auto it = h->m.tensors.find(tensor_id);
    if (it == h->m.tensors.end()) return -1;
    *data = it->second.data();
    return (int64_t)it->second.size();
}

const char* spt_parakeet_onnx_piece(const spt_pk_onnx* h, int32_t token_id) {
    if (!h || token_id < 0 || (size_t)token_id >= h->m.pieces.size()) return nullptr;
    return h->m.pieces[token_id].c_str();
}

void spt_parakeet_onnx_close(spt_pk_onnx* h) { delete h; }

const char* spt_parakeet_last_error(const spt_pk_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

spt_status spt_parakeet_info(const spt_pk_ctx* ctx, spt_pk_model_info* info) {
    if (!ctx || !info) return SPT_ERR_INVALID_ARG;
    const spt::PkDims& d = ctx->eng->dims();
    info->n_mels = d.n_mels; info->d = d.d; info->n_layers = d.n_layers; info->n_heads = d.n_heads; info->ff = d.ff;
    info->sub_ch = d.sub_ch; info->conv_k = d.conv_k; info->pred = d.pred; info->n_vocab = d.n_vocab;
    info->n_dur = d.n_dur;
    const int dt = ctx->eng->dtype();
    info->dtype = dt == spt::DT_F16 ? SPT_DTYPE_F16 : dt == spt::DT_BF16 ? SPT_DTYPE_BF16 : SPT_DTYPE_F32;
    info->max_batch = ctx->eng->max_batch();
    info->max_samples = ctx->eng->max_samples();
    info->reserved0 = 0;
    info->weight_bytes = ctx->eng->weight_bytes();
    info->workspace_bytes = ctx->eng->workspace_bytes();
    return SPT_OK;
}

spt_status spt_parakeet_tensor_numel(const spt_pk_ctx* ctx, int32_t tensor_id, int64_t* n) {
    if (!ctx || !n) return SPT_ERR_INVALID_ARG;
    *n = ctx->eng->tensor_numel(tensor_id);
    return *n < 0 ? SPT_ERR_INVALID_ARG : SPT_OK;
}

spt_status spt_parakeet_set_tensor(spt_pk_ctx* ctx, int32_t tensor_id, const float* data, int64_t n) {
    if (!ctx || !data) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        ctx->eng->set_tensor(tensor_id, data, n);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_set_vocab(spt_pk_ctx* ctx, const char* const* pieces, int32_t n) {
    if (!ctx || (n > 0 && !pieces) || n < 0) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n > 0 && n != ctx->eng->dims().n_vocab)
        return fail(ctx, SPT_ERR_INVALID_ARG, "vocabulary size differs from the model's n_vocab");
    std::vector<std::string> v;
    for (int32_t i = 0; i < n; ++i) v.push_back(pieces[i] ? pieces[i] : "");
    ctx->pieces.swap(v);
    return SPT_OK;
}

spt_status spt_parakeet_transcribe_batch(spt_pk_ctx* ctx, const float* const* pcm, const size_t* n_samples, size_t batch,
                                         const spt_pk_infer_params* params, spt_pk_result** out) {
    if (!ctx || !out || (batch && (!pcm || !n_samples))) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    spt_pk_infer_params dp;
    spt_parakeet_default_infer_params(&dp);
    if (!params) params = &dp;
    spt_status s = check_params(ctx, params);
    if (s != SPT_OK) return s;
    for (size_t u = 0; u < batch; ++u) {
        out[u] = nullptr;
        if (n_samples[u] && !pcm[u]) return fail(ctx, SPT_ERR_INVALID_ARG, "null pcm");
        if (n_samples[u] > (size_t)INT32_MAX / 2) return fail(ctx, SPT_ERR_INVALID_ARG, "utterance too long");
    }
    spt::ParakeetEngine& e = *ctx->eng;
    size_t longest = 0;
    for (size_t u = 0; u < batch; ++u) longest = std::max(longest, n_samples[u]);
    try {
        if (longest > (size_t)e.max_samples() && longest <= 16000u * 1200u)
            e.reserve_samples((int)longest, kMaxGrowBytes);  // false: the chunked fallback below
    } catch (const std::exception& ex) {
        return fail(ctx, classify(ex), ex.what());
    }
    const int cs = e.max_samples();
    struct Chunk { size_t utt; int idx; const float* p; int n; };
    std::vector<Chunk> ch;
    std::vector<int> nch(batch, 0);
    for (size_t u = 0; u < batch; ++u)
        for (size_t o = 0; o < n_samples[u]; o += cs) {
            ch.push_back(Chunk{u, nch[u]++, pcm[u] + o, (int)std::min<size_t>(cs, n_samples[u] - o)});
        }
    try {
        std::vector<spt::PkUtt> acc(batch);
        const int fpc = cs / kFrameSamples;  // encoder frames per full chunk
        for (size_t g0 = 0; g0 < ch.size(); g0 += e.max_batch()) {
            const int B = (int)std::min<size_t>(e.max_batch(), ch.size() - g0);
            std::vector<const float*> ptr(B);
            std::vector<int> ns(B);
            for (int b = 0; b < B; ++b) { ptr[b] = ch[g0 + b].p; ns[b] = ch[g0 + b].n; }
            std::vector<spt::PkUtt> res;
            e.transcribe_host(ptr.data(), ns.data(), B, params->max_symbols, &res);
            for (int b = 0; b < B; ++b) {
                const Chunk& k = ch[g0 + b];
                spt::PkUtt& a = acc[k.utt];
                const spt::PkUtt& r = res[b];
                for (size_t i = 0; i < r.tok.size(); ++i) {
                    a.tok.push_back(r.tok[i]);
                    a.frame.push_back(r.frame[i] + k.idx * fpc);
                    a.top1.push_back(r.top1[i]);
                    a.top2.push_back(r.top2[i]);
                }
            }
        }
        for (size_t u = 0; u < batch; ++u) {
            out[u] = make_result(ctx, acc[u], nch[u], params->timestamp_granularity);
            if (!out[u]) {
                for (size_t v = 0; v < u; ++v) { spt_parakeet_result_free(out[v]); out[v] = nullptr; }
                return fail(ctx, SPT_ERR_OOM, "host allocation failed");
            }
        }
        return SPT_OK;
    } catch (const std::exception& ex) {
        return fail(ctx, classify(ex), ex.what());
    }
}

spt_status spt_parakeet_transcribe(spt_pk_ctx* ctx, const float* pcm16k, size_t n_samples,
                                   const spt_pk_infer_params* params, spt_pk_result** out) {
    if (!ctx || !out) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n_samples && !pcm16k) return fail(ctx, SPT_ERR_INVALID_ARG, "null pcm");
    return spt_parakeet_transcribe_batch(ctx, &pcm16k, &n_samples, 1, params, out);
}

spt_status spt_parakeet_transcribe_batch_device(spt_pk_ctx* ctx, const float* pcm_dev, size_t stride,
                                                const size_t* n_samples, size_t batch,
                                                const spt_pk_infer_params* params, spt_pk_result** out) {
    if (!ctx || !out || !pcm_dev || !n_samples || batch == 0) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    spt::ParakeetEngine& e = *ctx->eng;
    if (batch > (size_t)e.max_batch()) return fail(ctx, SPT_ERR_INVALID_ARG, "batch exceeds max_batch");
    spt_pk_infer_params dp;
    spt_parakeet_default_infer_params(&dp);
    if (!params) params = &dp;
    spt_status s = check_params(ctx, params);
    if (s != SPT_OK) return s;
    std::vector<int> ns(batch);
    size_t longest = 0;
    for (size_t b = 0; b < batch; ++b) {
        out[b] = nullptr;
        if (n_samples[b] > 16000u * 1200u) return fail(ctx, SPT_ERR_INVALID_ARG, "utterance longer than 20 minutes");
        if (batch > 1 && n_samples[b] > stride) return fail(ctx, SPT_ERR_INVALID_ARG, "utterance longer than the device stride");
        ns[b] = (int)n_samples[b];
        longest = std::max(longest, n_samples[b]);
    }
    try {
        if (longest > (size_t)e.max_samples() && !e.reserve_samples((int)longest, kMaxGrowBytes))
            return fail(ctx, SPT_ERR_OOM, "no device room to decode an utterance this long in one pass");
        std::vector<spt::PkUtt> res;
        e.transcribe_device(pcm_dev, (int64_t)stride, ns.data(), (int)batch, params->max_symbols, &res);
        for (size_t b = 0; b < batch; ++b) {
            out[b] = make_result(ctx, res[b], 1, params->timestamp_granularity);
            if (!out[b]) {
                for (size_t v = 0; v < b; ++v) { spt_parakeet_result_free(out[v]); out[v] = nullptr; }
                return fail(ctx, SPT_ERR_OOM, "host allocation failed");
            }
        }
        return SPT_OK;
    } catch (const std::exception& ex) {
        return fail(ctx, classify(ex), ex.what());
    }
}

void spt_parakeet_result_free(spt_pk_result* r) {
    if (!r) return;
    for (int32_t i = 0; i < r->n_segments && r->segments; ++i) free(r->segments[i].text);
    free(r->segments);
    free(r->text);
    free(r->tokens);
    free(r->frames);
    free(r->logit);
    free(r->runner_up);
    free(r);
}

spt_status spt_parakeet_get_timings(const spt_pk_ctx* ctx, spt_pk_timings* t) {
    if (!ctx || !t) return SPT_ERR_INVALID_ARG;
    const spt::PkTimings& m = ctx->eng->timings();
    t->mel_ms = m.mel_ms; t->encoder_ms = m.encoder_ms; t->decode_ms = m.decode_ms; t->total_ms = m.total_ms;
    t->h2d_ms = m.h2d_ms; t->n_steps = m.n_steps; t->batch = m.batch; t->enc_frames = m.enc_frames;
    t->reserved0 = 0;
    return SPT_OK;
}

spt_status spt_parakeet_profile_encoder(spt_pk_ctx* ctx, int32_t iters, double* ms, int32_t n) {
    static_assert(SPT_PK_STAGE_COUNT == spt::PK_ST_COUNT, "stage classes");
    if (!ctx || !ms || n < SPT_PK_STAGE_COUNT) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument or n too small");
    try {
        ctx->eng->profile_encoder(iters, ms);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_debug_mel(spt_pk_ctx* ctx, const float* pcm16k, size_t n_samples, float* out) {
    if (!ctx || !out || (n_samples && !pcm16k)) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    if (n_samples > (size_t)ctx->eng->max_samples()) return fail(ctx, SPT_ERR_INVALID_ARG, "longer than max_seconds");
    try {
        ctx->eng->debug_mel(pcm16k, (int)n_samples, out);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_debug_encode(spt_pk_ctx* ctx, const float* mel, int32_t T, float* out) {
    if (!ctx || !mel || !out) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        ctx->eng->debug_encode(mel, T, out);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_debug_last_encoder(spt_pk_ctx* ctx, int32_t b, float* out, int32_t* T3) {
    if (!ctx || !out || !T3) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        *T3 = ctx->eng->debug_last_encoder(b, out);
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_debug_decode(spt_pk_ctx* ctx, const float* enc, int32_t T3, int32_t max_symbols,
                                     spt_pk_result** out) {
    if (!ctx || !enc || !out) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    try {
        spt::PkUtt r;
        ctx->eng->debug_decode(enc, T3, max_symbols, &r);
        *out = make_result(ctx, r, 1, SPT_PK_TS_TOKEN);
        return *out ? SPT_OK : fail(ctx, SPT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

spt_status spt_parakeet_debug_weight_checksum(spt_pk_ctx* ctx, int32_t tensor_id, double* out2) {
    if (!ctx || !out2) return fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    try {
        if (!ctx->eng->has_tensor(tensor_id)) return fail(ctx, SPT_ERR_INVALID_ARG, "unknown tensor id");
        if (!ctx->eng->debug_weight_checksum(tensor_id, out2))
            return fail(ctx, SPT_ERR_UNSUPPORTED, "tensor is stored transposed inside a shared block");
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(ctx, classify(e), e.what());
    }
}

}  // extern "C"
