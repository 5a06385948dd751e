// engine.cpp -- device-resident Whisper engine: weights, static memory plan,
// the mel -> encoder -> cross-KV -> greedy decode pipeline, hipGraph decode steps.
//
// Reference path replaced: WhisperEngine::transcribe_samples -> whisper_full
// (/root/reference/src-tauri/src/managers/transcription.rs:494-503), i.e.
// whisper.cpp's log_mel_spectrogram, whisper_encode_internal (conv stem +
// encoder + cross K/V) and the whisper_decode_internal / whisper_process_logits
// / whisper_sample_token loop, for the greedy, fixed-language, no-timestamp
// protocol of BASELINE.md.
#include "engine.h"
#include "ggml_file.h"

#include <cstdio>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <cstdlib>
#include <sstream>
#include <stdexcept>

#include "common.h"

namespace spt {

bool parse_synthetic_spec(const std::string& spec, ModelDims* dm, uint64_t* seed, std::string* err) {
    const std::string pfx = "synthetic:";
    if (spec.compare(0, pfx.size(), pfx) != 0) return false;
    std::vector<std::string> parts;
    std::stringstream ss(spec.substr(pfx.size()));
    std::string tok;
    while (std::getline(ss, tok, ':')) parts.push_back(tok);
    if (parts.empty()) { *err = "empty synthetic spec"; return true; }
    struct Cfg { const char* name; int n_mels, d, h, ne, nd, V; };
    static const Cfg cfgs[] = {
        {"tiny.en", 80, 384, 6, 4, 4, 51864},     {"tiny", 80, 384, 6, 4, 4, 51865},
        {"base.en", 80, 512, 8, 6, 6, 51864},     {"base", 80, 512, 8, 6, 6, 51865},
        {"small.en", 80, 768, 12, 12, 12, 51864}, {"small", 80, 768, 12, 12, 12, 51865},
        {"medium.en", 80, 1024, 16, 24, 24, 51864}, {"medium", 80, 1024, 16, 24, 24, 51865},
        {"large-v3", 128, 1280, 20, 32, 32, 51866}, {"large-v3-turbo", 128, 1280, 20, 32, 4, 51866},
    };
    bool found = false;
    for (const Cfg& c : cfgs)
        if (parts[0] == c.name) {
            dm->name = c.name;
            dm->n_mels = c.n_mels; dm->d = c.d; dm->n_head = c.h; dm->n_enc = c.ne; dm->n_dec = c.nd;
            dm->n_vocab = c.V;
            found = true;
        }
    if (!found) { *err = "unknown synthetic model '" + parts[0] + "'"; return true; }
    for (size_t i = 1; i < parts.size(); ++i) {
        const std::string& p = parts[i];
        const size_t eq = p.find('=');
        if (eq == std::string::npos) { *err = "bad option '" + p + "'"; return true; }
        const std::string k = p.substr(0, eq), v = p.substr(eq + 1);
        char* end = nullptr;
        const unsigned long long x = strtoull(v.c_str(), &end, 10);
        if (!end || *end) { *err = "bad value in '" + p + "'"; return true; }
        if (k == "enc") dm->n_enc = (int)x;
        else if (k == "dec") dm->n_dec = (int)x;
        else if (k == "seed") *seed = (uint64_t)x;
        else { *err = "unknown option '" + k + "'"; return true; }
    }
    if (dm->n_enc < 0 || dm->n_dec < 1 || dm->n_enc > 64 || dm->n_dec > 64) *err = "layer count out of range";
    return true;
}

// ----------------------------------------------------------------------------- helpers
namespace {
int fanin_exp(int K) { return (int)floor(log2(sqrt(3.0 / (double)K)) + 0.5); }

struct Carver {
    char* base;
    int64_t off = 0;
    void* take(int64_t bytes) {
        off = (off + 255) & ~(int64_t)255;
        void* p = base ? base + off : nullptr;
        off += bytes;
        return p;
    }
};
}  // namespace

void Engine::select() const { HIP_CHECK(hipSetDevice(dev_)); }

Engine::Engine(const ModelDims& dm, int dtype, int device, int max_batch, uint64_t seed, const GgmlFile* src,
               bool external_weights)
    : dm_(dm), dt_(dtype), dev_(device), max_batch_(max_batch), seed_(seed) {
    if (dm_.d % 128 || dm_.d / 64 != dm_.n_head) throw std::runtime_error("unsupported model width");
    if (max_batch_ < 1 || max_batch_ > 64) throw std::runtime_error("max_batch must be in 1..64");
    if (dt_ == DT_F32 && dm_.d > 1024)  // LayerNorm-prologue GEMVs stage <= 16 f32 super-steps
        throw std::runtime_error("the f32 engine supports model widths up to 1024 (tiny..medium); load " +
                                 std::to_string(dm_.d) + "-wide models in bf16");
    esz_ = dt_ == DT_BF16 ? 2 : 4;
    cp_ = ((dm_.n_mels + 63) / 64) * 64;
    if ((3 * cp_ * esz_) % 128) cp_ = ((dm_.n_mels + 127) / 128) * 128;
    if (const char* g = getenv("SPT_DECODE_GROUPS")) n_groups_ = std::max(1, std::min(4, atoi(g)));
    if (const char* v = getenv("SPT_XATTN_SPLIT")) xsplit_ = std::max(1, std::min(4, atoi(v)));
    // cross-attention key split: fixed per engine (never per batch).  The fc2 K split (2; r1
    // exp14 measured 2 slightly faster per layer than 4: the next QKV LayerNorm prologue sums
    // fewer slabs) is fixed per engine too; the pending-slab count a LayerNorm prologue sums is
    // a kernel template constant.
    select();
    HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    ev_.resize(12);  // 0-1 mel, 2-5 window / encoder / cross K/V, 6-7 decode, 8-9 a beam step, 10-11 H2D
    for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
    enc_st_.assign(kEncGroupsMax - 1, nullptr);
    for (auto& s : enc_st_) HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    enc_ev_.assign(kEncGroupsMax, nullptr);
    for (auto& e : enc_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // a decoder pass stages at most max_rows_ rows in its LayerNorm GEMVs' LDS images; a batch
    // above that is decoded as several groups (each sized for the whole batch, re-sliced per call)
    max_rows_ = gemv_max_image_rows(dt_, dm_.d);
    groups_.resize(std::max(n_groups_, cdiv(max_batch_, max_rows_)));
    for (auto& g : groups_) {
        HIP_CHECK(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&g.ev, hipEventDisableTiming));
    }
    try {
        gemv_prepare(dt_);
        gemm_prepare();  // > 64 KiB LDS attributes on this device, before any capture
        alloc_weights();
        if (external_weights) {
            // filled later by import_weights; clear it so a premature use reads zeros, not garbage
            HIP_CHECK(hipMemsetAsync(warena_, 0, wbytes_, st_));
        } else if (src) {
            load_ggml(*src);
        } else {
            generate_weights();
        }
        weights_ready_ = !external_weights;
        upload_tables(src ? &src->mel_filters() : nullptr);
        alloc_workspace();
        HIP_CHECK(hipStreamSynchronize(st_));
    } catch (...) {
        release();  // a throwing constructor runs no destructor
        throw;
    }
}

Engine::~Engine() { release(); }

void Engine::release() {
    (void)hipSetDevice(dev_);
    if (st_) (void)hipStreamSynchronize(st_);
    for (auto& g : groups_) {
        if (g.st) (void)hipStreamSynchronize(g.st);
        for (auto& kv : g.graphs) (void)hipGraphExecDestroy(kv.second);
        if (g.ev) (void)hipEventDestroy(g.ev);
        if (g.st) (void)hipStreamDestroy(g.st);
    }
    for (auto& kv : enc_graphs_) (void)hipGraphExecDestroy(kv.second);
    enc_graphs_.clear();
    for (auto& s : enc_st_)
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    enc_st_.clear();
    for (auto& e : enc_ev_)
        if (e) (void)hipEventDestroy(e);
    enc_ev_.clear();
    if (warena_) (void)hipFree(warena_);
    if (aarena_) (void)hipFree(aarena_);
    if (kvtmp_) (void)hipFree(kvtmp_);
    for (void* p : {(void*)upcm_, (void*)umel_, (void*)uinfo_})
        if (p) (void)hipFree(p);
    upcm_ = umel_ = nullptr;
    uinfo_ = nullptr;
    upcm_cap_ = umel_cap_ = 0;
    uinfo_cap_ = 0;
    for (void* p : {(void*)hann_, (void*)sinv_, (void*)cosv_, (void*)filt_, (void*)grp_})
        if (p) (void)hipFree(p);
    for (auto& e : ev_) (void)hipEventDestroy(e);
    for (auto& e : probe_ev_) (void)hipEventDestroy(e);
    probe_ev_.clear();
    if (st_) (void)hipStreamDestroy(st_);
    groups_.clear();
    ev_.clear();
    warena_ = aarena_ = nullptr;
    kvtmp_ = nullptr;
    hann_ = sinv_ = cosv_ = filt_ = nullptr;
    grp_ = nullptr;
    st_ = nullptr;
}

// ----------------------------------------------------------------------------- weights
void Engine::require_weights() const {
    if (!weights_ready_)
        throw std::runtime_error("weights not loaded: the context was created with SPT_MODEL_WEIGHTS_EXTERNAL and "
                                 "spt_weights_import has not been called");
}

void Engine::export_weights(void* dev_dst, int64_t bytes) {
    require_weights();
    if (!dev_dst || bytes != wbytes_)
        throw std::runtime_error("weight export: expected " + std::to_string(wbytes_) + " bytes, got " +
                                 std::to_string(bytes));
    select();
    HIP_CHECK(hipMemcpyAsync(dev_dst, warena_, (size_t)wbytes_, hipMemcpyDeviceToDevice, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
}

void Engine::import_weights(const void* dev_src, int64_t bytes) {
    if (!dev_src || bytes != wbytes_)
        throw std::runtime_error("weight import: expected " + std::to_string(wbytes_) + " bytes (this model and dtype), got " +
                                 std::to_string(bytes));
    select();
    HIP_CHECK(hipMemcpyAsync(warena_, dev_src, (size_t)wbytes_, hipMemcpyDeviceToDevice, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    weights_ready_ = true;
}

void Engine::commit_weights() {
    select();
    HIP_CHECK(hipDeviceSynchronize());  // the writer may have used any stream of this device
    weights_ready_ = true;
}

void Engine::alloc_weights() {
    const int64_t d = dm_.d, dd = d * d, V = dm_.n_vocab, L = dm_.n_dec;
    enc_.resize(dm_.n_enc);
    dec_.resize(dm_.n_dec);
    for (int pass = 0; pass < 2; ++pass) {
        Carver c{pass ? warena_ : nullptr};
        auto W = [&](int64_t n) { return c.take(n * esz_); };
        auto F = [&](int64_t n) { return (float*)c.take(n * 4); };
        conv1_w_ = W(d * 3 * cp_); conv1_b_ = F(d);
        conv2_w_ = W(dd * 3); conv2_b_ = F(d);
        enc_pos_ = F((int64_t)dm_.n_audio_ctx * d);
        lnp_w_ = F(d); lnp_b_ = F(d);
        for (auto& e : enc_) {
            e.ln1_w = F(d); e.ln1_b = F(d); e.qkv_w = W(3 * dd); e.qkv_b = F(3 * d); e.o_w = W(dd); e.o_b = F(d);
            e.ln2_w = F(d); e.ln2_b = F(d); e.fc1_w = W(4 * dd); e.fc1_b = F(4 * d); e.fc2_w = W(4 * dd); e.fc2_b = F(d);
        }
        ckv_w_ = W(L * 2 * dd); ckv_b_ = F(L * 2 * d);
        tok_emb_ = W(V * d); dec_pos_ = F((int64_t)dm_.n_text_ctx * d); lnf_w_ = F(d); lnf_b_ = F(d);
        for (auto& e : dec_) {
            e.ln1_w = F(d); e.ln1_b = F(d); e.qkv_w = W(3 * dd); e.qkv_b = F(3 * d); e.so_w = W(dd); e.so_b = F(d);
            e.ln2_w = F(d); e.ln2_b = F(d); e.cq_w = W(dd); e.cq_b = F(d); e.co_w = W(dd); e.co_b = F(d);
            e.ln3_w = F(d); e.ln3_b = F(d); e.fc1_w = W(4 * dd); e.fc1_b = F(4 * d); e.fc2_w = W(4 * dd); e.fc2_b = F(d);
        }
        if (!pass) {
            wbytes_ = c.off;
            if (hipMalloc(&warena_, wbytes_) != hipSuccess) {
                warena_ = nullptr;
                throw std::runtime_error("out of device memory for weights (" + std::to_string(wbytes_) + " B)");
            }
        }
    }
}

void Engine::generate_weights() {
    const int64_t d = dm_.d, dd = d * d;
    auto reg = [&](int tid, void* p, int64_t n, int dt) { tref_[tid] = TRef{p, n, dt}; };
    auto genw = [&](void* p, int64_t n, int tid, int kind, int e) {  // dtype storage
        gen_weights(dt_, p, n, seed_, (uint32_t)tid, kind, e, st_);
        reg(tid, p, n, dt_);
    };
    auto genf = [&](float* p, int64_t n, int tid, int kind, int e) {  // f32 storage
        gen_weights(DT_F32, p, n, seed_, (uint32_t)tid, kind, e, st_);
        reg(tid, p, n, DT_F32);
    };
    auto at = [&](void* p, int64_t elems) { return (void*)((char*)p + elems * esz_); };
    gen_conv_weights(dt_, conv1_w_, (int)d, dm_.n_mels, cp_, seed_, 1, fanin_exp(3 * dm_.n_mels), st_);
    reg(1, conv1_w_, d * 3 * cp_, dt_);
    genf(conv1_b_, d, 2, WK_BIAS, -5);
    gen_conv_weights(dt_, conv2_w_, (int)d, (int)d, (int)d, seed_, 3, fanin_exp(3 * (int)d), st_);
    reg(3, conv2_w_, dd * 3, dt_);
    genf(conv2_b_, d, 4, WK_BIAS, -5);
    genf(lnp_w_, d, 5, WK_LNW, -3);
    genf(lnp_b_, d, 6, WK_LNB, -4);
    {  // whisper sinusoids(1500, d), double precision like the oracle
        std::vector<float> pe((size_t)dm_.n_audio_ctx * d);
        const int half = (int)d / 2;
        const double inc = log(10000.0) / (double)(half - 1);
        for (int t = 0; t < dm_.n_audio_ctx; ++t)
            for (int i = 0; i < half; ++i) {
                const double s = (double)t * exp(-inc * (double)i);
                pe[(size_t)t * d + i] = (float)sin(s);
                pe[(size_t)t * d + half + i] = (float)cos(s);
            }
        HIP_CHECK(hipMemcpy(enc_pos_, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
        reg(7, enc_pos_, (int64_t)pe.size(), DT_F32);
    }
    for (int l = 0; l < dm_.n_enc; ++l) {
        EncL& e = enc_[l];
        const int b = 100 + 32 * l;
        genf(e.ln1_w, d, b + 0, WK_LNW, -3);
        genf(e.ln1_b, d, b + 1, WK_LNB, -4);
        genw(at(e.qkv_w, 0), dd, b + 2, WK_MAT, fanin_exp((int)d));
        genf(e.qkv_b, d, b + 3, WK_BIAS, -5);
        genw(at(e.qkv_w, dd), dd, b + 4, WK_MAT, fanin_exp((int)d));
        fill_f32(e.qkv_b + d, d, 0.0f, st_);
        genw(at(e.qkv_w, 2 * dd), dd, b + 5, WK_MAT, fanin_exp((int)d));
        genf(e.qkv_b + 2 * d, d, b + 6, WK_BIAS, -5);
        genw(e.o_w, dd, b + 7, WK_MAT, fanin_exp((int)d));
        genf(e.o_b, d, b + 8, WK_BIAS, -5);
        genf(e.ln2_w, d, b + 9, WK_LNW, -3);
        genf(e.ln2_b, d, b + 10, WK_LNB, -4);
        genw(e.fc1_w, 4 * dd, b + 11, WK_MAT, fanin_exp((int)d));
        genf(e.fc1_b, 4 * d, b + 12, WK_BIAS, -5);
        genw(e.fc2_w, 4 * dd, b + 13, WK_MAT, fanin_exp(4 * (int)d));
        genf(e.fc2_b, d, b + 14, WK_BIAS, -5);
    }
    genw(tok_emb_, (int64_t)dm_.n_vocab * d, 10, WK_TOK, -2);
    genf(dec_pos_, (int64_t)dm_.n_text_ctx * d, 11, WK_DPOS, 0);
    genf(lnf_w_, d, 12, WK_LNW, -3);
    genf(lnf_b_, d, 13, WK_LNB, -4);
    for (int l = 0; l < dm_.n_dec; ++l) {
        DecL& e = dec_[l];
        const int b = 5000 + 32 * l;
        genf(e.ln1_w, d, b + 0, WK_LNW, -3);
        genf(e.ln1_b, d, b + 1, WK_LNB, -4);
        genw(at(e.qkv_w, 0), dd, b + 2, WK_MAT, fanin_exp((int)d));
        genf(e.qkv_b, d, b + 3, WK_BIAS, -5);
        genw(at(e.qkv_w, dd), dd, b + 4, WK_MAT, fanin_exp((int)d));
        fill_f32(e.qkv_b + d, d, 0.0f, st_);
        genw(at(e.qkv_w, 2 * dd), dd, b + 5, WK_MAT, fanin_exp((int)d));
        genf(e.qkv_b + 2 * d, d, b + 6, WK_BIAS, -5);
        genw(e.so_w, dd, b + 7, WK_MAT, fanin_exp((int)d));
        genf(e.so_b, d, b + 8, WK_BIAS, -5);
        genf(e.ln2_w, d, b + 9, WK_LNW, -3);
        genf(e.ln2_b, d, b + 10, WK_LNB, -4);
        genw(e.cq_w, dd, b + 11, WK_MAT, fanin_exp((int)d));
        genf(e.cq_b, d, b + 12, WK_BIAS, -5);
        genw(at(ckv_w_, (2 * l) * dd), dd, b + 13, WK_MAT, fanin_exp((int)d));
        fill_f32(ckv_b_ + (2 * l) * d, d, 0.0f, st_);
        genw(at(ckv_w_, (2 * l + 1) * dd), dd, b + 14, WK_MAT, fanin_exp((int)d));
        genf(ckv_b_ + (2 * l + 1) * d, d, b + 15, WK_BIAS, -5);
        genw(e.co_w, dd, b + 16, WK_MAT, fanin_exp((int)d));
        genf(e.co_b, d, b + 17, WK_BIAS, -5);
        genf(e.ln3_w, d, b + 18, WK_LNW, -3);
        genf(e.ln3_b, d, b + 19, WK_LNB, -4);
        genw(e.fc1_w, 4 * dd, b + 20, WK_MAT, fanin_exp((int)d));
        genf(e.fc1_b, 4 * d, b + 21, WK_BIAS, -5);
        genw(e.fc2_w, 4 * dd, b + 22, WK_MAT, fanin_exp(4 * (int)d));
        genf(e.fc2_b, d, b + 23, WK_BIAS, -5);
    }
    HIP_CHECK(hipGetLastError());
}

// ----------------------------------------------------------------------------- ggml models
bool ggml_dims(const GgmlFile& f, ModelDims* dm, std::string* err) {
    const GgmlHparams& h = f.hparams();
    if (h.n_audio_state != h.n_text_state) { *err = "encoder and decoder widths differ"; return false; }
    if (h.n_audio_head != h.n_text_head || h.n_audio_state != 64 * h.n_audio_head) {
        *err = "unsupported head layout (head dim must be 64)";
        return false;
    }
    if (h.n_audio_ctx != 1500 || h.n_text_ctx != 448) { *err = "unsupported context sizes"; return false; }
    if (h.n_mels != 80 && h.n_mels != 128) { *err = "unsupported n_mels " + std::to_string(h.n_mels); return false; }
    if (f.n_mel_filters() != h.n_mels || f.n_fft() != 201) { *err = "mel filterbank is not [n_mels][201]"; return false; }
    if (h.n_audio_layer < 1 || h.n_text_layer < 1 || h.n_vocab < 51864) { *err = "bad layer count or vocabulary"; return false; }
    dm->name = "ggml";
    dm->n_mels = h.n_mels;
    dm->d = h.n_audio_state;
    dm->n_head = h.n_audio_head;
    dm->n_enc = h.n_audio_layer;
    dm->n_dec = h.n_text_layer;
    dm->n_vocab = h.n_vocab;
    dm->n_audio_ctx = h.n_audio_ctx;
    dm->n_text_ctx = h.n_text_ctx;
    return true;
}

// whisper.cpp whisper_model_load's tensor names -> the engine arena.  Matrices (and the token
// embedding, conv kernels) are stored in the engine dtype, everything else in f32; q/k/v are
// fused into one [3d][d] matrix (the key has no bias: zeros), each decoder layer's cross K/V
// projection into ckv_w_ rows [2l d, 2l d + 2d).  Conv kernels are re-laid [d][C][3] ->
// [d][3][Cp] (Cp = padded mel channels) for the implicit-GEMM convolution.  Tensor ids match
// generate_weights() so the checksum probes address both kinds of model alike.
void Engine::load_ggml(const GgmlFile& f) {
    const int64_t d = dm_.d, dd = d * d;
    std::vector<std::pair<const GgmlTensor*, std::string>> used;
    auto need = [&](const std::string& name, int64_t n) -> const GgmlTensor* {
        const GgmlTensor* t = f.find(name);
        if (!t) throw std::runtime_error("model file lacks tensor " + name);
        if (t->numel() != n)
            throw std::runtime_error("tensor " + name + " has " + std::to_string(t->numel()) + " elements, expected " +
                                     std::to_string(n));
        return t;
    };
    size_t stage_bytes = 0;
    struct Staging {
        void* p = nullptr;
        ~Staging() { if (p) (void)hipFree(p); }
    } staging;
    for (int pass = 0; pass < 2; ++pass) {  // pass 0 sizes the staging buffer, pass 1 loads
        if (pass) HIP_CHECK(hipMalloc(&staging.p, std::max<size_t>(stage_bytes, 256)));
        void* stage = staging.p;
        auto put = [&](const std::string& name, int64_t n, void* dst, int dt, int tid) {
            const GgmlTensor* t = need(name, n);
            if (!pass) { stage_bytes = std::max(stage_bytes, t->nbytes); return; }
            HIP_CHECK(hipMemcpyAsync(stage, t->data, t->nbytes, hipMemcpyHostToDevice, st_));
            ggml_dequant(t->type, stage, n, dt, dst, st_);
            HIP_CHECK(hipStreamSynchronize(st_));  // the staging buffer is reused by the next tensor
            tref_[tid] = TRef{dst, n, dt};
        };
        auto putf = [&](const std::string& name, int64_t n, float* dst, int tid) { put(name, n, dst, DT_F32, tid); };
        auto putw = [&](const std::string& name, int64_t n, void* dst, int tid) { put(name, n, dst, dt_, tid); };
        auto at = [&](void* p, int64_t elems) { return (void*)((char*)p + elems * esz_); };
        auto conv = [&](const std::string& name, int C, int Cp, void* dst, int tid) {
            const GgmlTensor* t = need(name, d * C * 3);
            if (!pass) return;
            std::vector<float> src((size_t)t->numel());
            if (!ggml_dequant_host(t->type, t->data, t->numel(), src.data()))
                throw std::runtime_error("unsupported ggml type for " + name);
            std::vector<float> lay((size_t)d * 3 * Cp, 0.0f);
            for (int64_t n = 0; n < d; ++n)
                for (int c = 0; c < C; ++c)
                    for (int j = 0; j < 3; ++j) lay[((size_t)n * 3 + j) * Cp + c] = src[((size_t)n * C + c) * 3 + j];
            if (dt_ == DT_BF16) {
                std::vector<bf16> h(lay.size());
                for (size_t i = 0; i < lay.size(); ++i) h[i] = f2bf(lay[i]);
                HIP_CHECK(hipMemcpy(dst, h.data(), h.size() * 2, hipMemcpyHostToDevice));
            } else {
                HIP_CHECK(hipMemcpy(dst, lay.data(), lay.size() * 4, hipMemcpyHostToDevice));
            }
            tref_[tid] = TRef{dst, (int64_t)lay.size(), dt_};
        };
        conv("encoder.conv1.weight", dm_.n_mels, cp_, conv1_w_, 1);
        putf("encoder.conv1.bias", d, conv1_b_, 2);
        conv("encoder.conv2.weight", (int)d, (int)d, conv2_w_, 3);
        putf("encoder.conv2.bias", d, conv2_b_, 4);
        putf("encoder.ln_post.weight", d, lnp_w_, 5);
        putf("encoder.ln_post.bias", d, lnp_b_, 6);
        putf("encoder.positional_embedding", (int64_t)dm_.n_audio_ctx * d, enc_pos_, 7);
        for (int l = 0; l < dm_.n_enc; ++l) {
            EncL& e = enc_[l];
            const int b = 100 + 32 * l;
            const std::string p = "encoder.blocks." + std::to_string(l) + ".";
            putf(p + "attn_ln.weight", d, e.ln1_w, b + 0);
            putf(p + "attn_ln.bias", d, e.ln1_b, b + 1);
            putw(p + "attn.query.weight", dd, at(e.qkv_w, 0), b + 2);
            putf(p + "attn.query.bias", d, e.qkv_b, b + 3);
            putw(p + "attn.key.weight", dd, at(e.qkv_w, dd), b + 4);
            putw(p + "attn.value.weight", dd, at(e.qkv_w, 2 * dd), b + 5);
            putf(p + "attn.value.bias", d, e.qkv_b + 2 * d, b + 6);
            putw(p + "attn.out.weight", dd, e.o_w, b + 7);
            putf(p + "attn.out.bias", d, e.o_b, b + 8);
            putf(p + "mlp_ln.weight", d, e.ln2_w, b + 9);
            putf(p + "mlp_ln.bias", d, e.ln2_b, b + 10);
            putw(p + "mlp.0.weight", 4 * dd, e.fc1_w, b + 11);
            putf(p + "mlp.0.bias", 4 * d, e.fc1_b, b + 12);
            putw(p + "mlp.2.weight", 4 * dd, e.fc2_w, b + 13);
            putf(p + "mlp.2.bias", d, e.fc2_b, b + 14);
            if (pass) fill_f32(e.qkv_b + d, d, 0.0f, st_);
        }
        putw("decoder.token_embedding.weight", (int64_t)dm_.n_vocab * d, tok_emb_, 10);
        putf("decoder.positional_embedding", (int64_t)dm_.n_text_ctx * d, dec_pos_, 11);
        putf("decoder.ln.weight", d, lnf_w_, 12);
        putf("decoder.ln.bias", d, lnf_b_, 13);
        for (int l = 0; l < dm_.n_dec; ++l) {
            DecL& e = dec_[l];
            const int b = 5000 + 32 * l;
            const std::string p = "decoder.blocks." + std::to_string(l) + ".";
            putf(p + "attn_ln.weight", d, e.ln1_w, b + 0);
            putf(p + "attn_ln.bias", d, e.ln1_b, b + 1);
            putw(p + "attn.query.weight", dd, at(e.qkv_w, 0), b + 2);
            putf(p + "attn.query.bias", d, e.qkv_b, b + 3);
            putw(p + "attn.key.weight", dd, at(e.qkv_w, dd), b + 4);
            putw(p + "attn.value.weight", dd, at(e.qkv_w, 2 * dd), b + 5);
            putf(p + "attn.value.bias", d, e.qkv_b + 2 * d, b + 6);
            putw(p + "attn.out.weight", dd, e.so_w, b + 7);
            putf(p + "attn.out.bias", d, e.so_b, b + 8);
            putf(p + "cross_attn_ln.weight", d, e.ln2_w, b + 9);
            putf(p + "cross_attn_ln.bias", d, e.ln2_b, b + 10);
            putw(p + "cross_attn.query.weight", dd, e.cq_w, b + 11);
            putf(p + "cross_attn.query.bias", d, e.cq_b, b + 12);
            putw(p + "cross_attn.key.weight", dd, at(ckv_w_, (2 * l) * dd), b + 13);
            putw(p + "cross_attn.value.weight", dd, at(ckv_w_, (2 * l + 1) * dd), b + 14);
            putf(p + "cross_attn.value.bias", d, ckv_b_ + (2 * l + 1) * d, b + 15);
            putw(p + "cross_attn.out.weight", dd, e.co_w, b + 16);
            putf(p + "cross_attn.out.bias", d, e.co_b, b + 17);
            putf(p + "mlp_ln.weight", d, e.ln3_w, b + 18);
            putf(p + "mlp_ln.bias", d, e.ln3_b, b + 19);
            putw(p + "mlp.0.weight", 4 * dd, e.fc1_w, b + 20);
            putf(p + "mlp.0.bias", 4 * d, e.fc1_b, b + 21);
            putw(p + "mlp.2.weight", 4 * dd, e.fc2_w, b + 22);
            putf(p + "mlp.2.bias", d, e.fc2_b, b + 23);
            if (pass) {
                fill_f32(e.qkv_b + d, d, 0.0f, st_);
                fill_f32(ckv_b_ + (2 * l) * d, d, 0.0f, st_);
            }
        }
        if (pass) HIP_CHECK(hipStreamSynchronize(st_));
    }
}

void Engine::upload_tables(const std::vector<float>* filters) {
    // whisper_global_cache: sin/cos tables and periodic Hann from float(theta)
    std::vector<float> hann(400), sv(400), cv(400);
    for (int i = 0; i < 400; ++i) {
        const double theta = (2 * M_PI * i) / 400;
        sv[i] = sinf((float)theta);
        cv[i] = cosf((float)theta);
        hann[i] = (float)(0.5 * (1.0 - cosf((float)((2.0 * M_PI * i) / 400))));
    }
    // librosa / slaney mel filterbank (the filters whisper.cpp reads from the model file)
    const int nm = dm_.n_mels;
    auto hz2mel = [](double f) {
        const double lg = 27.0 / log(6.4);
        return f >= 1000.0 ? 15.0 + log(f / 1000.0) * lg : 3.0 * f / 200.0;
    };
    auto mel2hz = [](double m) {
        const double lg = log(6.4) / 27.0;
        return m >= 15.0 ? 1000.0 * exp(lg * (m - 15.0)) : 200.0 * m / 3.0;
    };
    std::vector<double> ff(nm + 2);
    const double mmin = hz2mel(0.0), mmax = hz2mel(8000.0);
    for (int i = 0; i < nm + 2; ++i) {
        double mm = mmin + (mmax - mmin) * i / (double)(nm + 1);
        if (i == nm + 1) mm = mmax;
        ff[i] = mel2hz(mm);
    }
    std::vector<float> filt((size_t)nm * 201);
    std::vector<int> grp(2 * nm);
    if (filters) filt = *filters;  // the model file's bank (ggml_dims checked [n_mels][201])
    for (int j = 0; j < nm; ++j) {
        const double en = 2.0 / (ff[j + 2] - ff[j]);
        int lo = -1, hi = -1;
        for (int k = 0; k < 201; ++k) {
            if (!filters) {
                const double fk = 8000.0 * k / 200.0;
                const double down = -(ff[j] - fk) / (ff[j + 1] - ff[j]);
                const double up = (ff[j + 2] - fk) / (ff[j + 2] - ff[j + 1]);
                double v = std::min(down, up);
                if (v < 0) v = 0;
                filt[(size_t)j * 201 + k] = (float)(v * en);
            }
            const float fv = filt[(size_t)j * 201 + k];
            if (fv != 0.0f) {
                if (lo < 0) lo = k;
                hi = k;
            }
        }
        if (lo < 0) { grp[2 * j] = 0; grp[2 * j + 1] = 0; }
        else {
            grp[2 * j] = lo < 200 ? lo / 4 : 50;
            grp[2 * j + 1] = (hi < 200 ? hi / 4 : 50) + 1;
        }
    }
    HIP_CHECK(hipMalloc(&hann_, 400 * 4));
    HIP_CHECK(hipMalloc(&sinv_, 400 * 4));
    HIP_CHECK(hipMalloc(&cosv_, 400 * 4));
    HIP_CHECK(hipMalloc(&filt_, filt.size() * 4));
    HIP_CHECK(hipMalloc(&grp_, grp.size() * 4));
    HIP_CHECK(hipMemcpy(hann_, hann.data(), 1600, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(sinv_, sv.data(), 1600, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(cosv_, cv.data(), 1600, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(filt_, filt.data(), filt.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(grp_, grp.data(), grp.size() * 4, hipMemcpyHostToDevice));
}

// ----------------------------------------------------------------------------- workspace
void Engine::alloc_workspace() {
    const int64_t B = max_batch_, d = dm_.d, T = dm_.n_audio_ctx, L = dm_.n_dec, ctx = dm_.n_text_ctx;
    const int64_t V = dm_.n_vocab, R = B * 4;
    for (int pass = 0; pass < 2; ++pass) {
        Carver c{pass ? aarena_ : nullptr};
        auto A = [&](int64_t n) { return c.take(n * esz_); };
        win_utt_ = (int*)c.take(B * 4);
        win_seek_ = (int*)c.take(B * 4);
        mel_in_ = A(B * MEL_ROWS * cp_);
        y1p_ = A(B * MEL_ROWS * d);
        x_ = (float*)c.take(B * T * d * 4);
        xn_ = A(B * T * d);
        qkv_ = A(B * T * 3 * d);
        ao_ = A(B * T * d);
        ff_ = A(B * T * 4 * d);
        enc_out_ = A(B * T * d);
        ckv_ = A(L * kv_layer_elems((int)B, dm_.n_head, (int)T));
        suppress_ = (uint32_t*)c.take((V / 32 + 1) * 4);
        suppress_lang_ = (uint32_t*)c.take((V / 32 + 1) * 4);
        scratch_ = (double*)c.take(64);
        for (DecGroup& g : groups_) {  // each group sized for the whole batch (groups are re-sliced per call)
            g.dx = (float*)c.take(R * d * 4);
            g.dq = A(R * d);
            g.dao = A(R * d);
            g.dff = A(R * 4 * d);
            g.skv = A(L * 2 * B * ctx * d);
            g.logits = (float*)c.take(B * V * 4);
            g.part = c.take(B * ((V + 15) / 16) * 16);
            g.arrive = (unsigned*)c.take(64);
            g.tok_in = (int*)c.take(R * 4);
            g.out_tok = (int*)c.take(B * ctx * 4);
            g.out_t1 = (float*)c.take(B * ctx * 4);
            g.out_t2 = (float*)c.take(B * ctx * 4);
            g.done = (int*)c.take(B * 4);
            g.forced = (int*)c.take(B * ctx * 4);
            g.ds = (DecState*)c.take(sizeof(DecState));
            g.dx2 = (float*)c.take(R * d * 4);
            g.pend = (float*)c.take((int64_t)kMaxPend * R * d * 4);
            g.xpart = (float*)c.take((int64_t)R * dm_.n_head * 8 * 66 * 4);
            g.seek = (int*)c.take(B * 4);
            g.seek_end = (int*)c.take(B * 4);
            g.ts_state = (int*)c.take(B * 16);
            g.ts_stat = (float*)c.take((int64_t)B * TS_CHUNKS * 6 * 4);
            g.beam_stat = (float*)c.take((int64_t)B * TS_CHUNKS * BEAM_STAT * 4);
            g.prm = (TsParams*)c.take(sizeof(TsParams));
            g.beam_row = (int*)c.take(B * 16);
            g.beam_step = (int*)c.take(64);
            g.beam_src = (int*)c.take(B * 4);
            g.cand_id = (int*)c.take(B * 8 * 4);
            g.cand_lp = (float*)c.take(B * 8 * 4);
            g.beam_tid = (int*)c.take(B * 4);
            g.kvrow = (int*)c.take(B * 4);
        }
        zero_ = (float*)c.take(R * d * 4);  // never written: the "no pending slab" operand
        if (!pass) {
            abytes_ = c.off;
            if (hipMalloc(&aarena_, abytes_) != hipSuccess) {
                aarena_ = nullptr;
                throw std::runtime_error("out of device memory for workspace (" + std::to_string(abytes_) + " B)");
            }
        }
    }
    // zero everything once: padding rows of the conv inputs stay zero forever
    HIP_CHECK(hipMemsetAsync(aarena_, 0, abytes_, st_));
}

// ----------------------------------------------------------------------------- pipeline
// ----------------------------------------------------------------------------- utterances
// a device buffer of at least `need` elements (grown by a quarter at a time; the old contents are
// not kept).  Only between calls: everything on the engine's streams has finished.
void Engine::ensure_capacity(void** p, int64_t* cap, int64_t need, size_t esz, const char* what) {
    if (need <= *cap) return;
    const int64_t want = std::max<int64_t>(need, *cap + *cap / 4);
    HIP_CHECK(hipDeviceSynchronize());
    if (*p) HIP_CHECK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, (size_t)want * esz) != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        throw std::runtime_error(std::string("out of device memory for ") + what + " (" +
                                 std::to_string((size_t)want * esz) + " B)");
    }
    *cap = want;
}

// whisper_pcm_to_mel of each whole utterance (k_mel.hip): pcm + pcm_off[u], n[u] samples each
void Engine::run_mel_utts(const float* pcm, const std::vector<int64_t>& pcm_off, const int* n, int U) {
    if (U < 1) throw std::runtime_error("no utterances");
    int64_t rows = 0;
    int max_rows = 0;
    uhost_.assign((size_t)U * 3, 0);  // pcm_off | row_off | n (as int64, unpacked on upload)
    for (int u = 0; u < U; ++u) {
        if (n[u] < 0) throw std::runtime_error("negative sample count");
        const int r = mel_rows(n[u]);
        uhost_[u] = pcm_off[u];
        uhost_[U + u] = rows;
        rows += r;
        max_rows = std::max(max_rows, r);
    }
    void* pm = umel_;
    ensure_capacity(&pm, &umel_cap_, std::max<int64_t>(rows, 1), (size_t)dm_.n_mels * 4, "the utterance log-mel");
    umel_ = (float*)pm;
    // info block: pcm_off [U] int64 | row_off [U] int64 | n [U] int | max [U] unsigned
    const int64_t info_bytes = (int64_t)U * 24;
    if (U > uinfo_cap_) {
        int64_t cap = uinfo_cap_ ? (int64_t)uinfo_cap_ * 24 : 0;
        void* pi = uinfo_;
        ensure_capacity(&pi, &cap, info_bytes, 1, "utterance descriptors");
        uinfo_ = (char*)pi;
        uinfo_cap_ = (int)(cap / 24);
    }
    mel_img_.assign((size_t)info_bytes, 0);
    memcpy(mel_img_.data(), uhost_.data(), (size_t)U * 16);
    for (int u = 0; u < U; ++u) memcpy(mel_img_.data() + (size_t)U * 16 + 4 * u, &n[u], 4);
    HIP_CHECK(hipMemcpyAsync(uinfo_, mel_img_.data(), (size_t)U * 20, hipMemcpyHostToDevice, st_));
    mu_.pcm_off = (const int64_t*)uinfo_;
    mu_.row_off = (const int64_t*)(uinfo_ + (size_t)U * 8);
    mu_.n = (const int*)(uinfo_ + (size_t)U * 16);
    umax_ = (unsigned*)(uinfo_ + (size_t)U * 20);
    un_.assign(n, n + U);
    HIP_CHECK(hipEventRecord(ev_[0], st_));
    MelTables t{hann_, sinv_, cosv_, filt_, grp_};
    mel_frames(pcm, mu_, U, max_rows, dm_.n_mels, t, umel_, umax_, st_);
    HIP_CHECK(hipEventRecord(ev_[1], st_));
    mel_pending_ = true;
    enc_E_ = 0;  // windows of an earlier set refer to its utterances
}

void Engine::load_utterances(const float* const* pcm, const int* n, int U) {
    select();
    require_weights();
    std::vector<int64_t> off(U);
    int64_t tot = 0;
    for (int u = 0; u < U; ++u) {
        if (n[u] < 0) throw std::runtime_error("negative sample count");
        if (n[u] > 0 && !pcm[u]) throw std::runtime_error("null pcm");
        off[u] = tot;
        tot += n[u];
    }
    void* pp = upcm_;
    ensure_capacity(&pp, &upcm_cap_, std::max<int64_t>(tot, 1), 4, "utterance PCM");
    upcm_ = (float*)pp;
    HIP_CHECK(hipEventRecord(ev_[10], st_));
    for (int u = 0; u < U; ++u)
        if (n[u] > 0)
            HIP_CHECK(hipMemcpyAsync(upcm_ + off[u], pcm[u], (size_t)n[u] * 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipEventRecord(ev_[11], st_));
    HIP_CHECK(hipEventSynchronize(ev_[11]));  // pageable sources: the caller may reuse them on return
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[10], ev_[11]));
    tm_.h2d_ms = ms;
    run_mel_utts(upcm_, off, n, U);
}

void Engine::load_utterances_device(const float* pcm_dev, int64_t stride, const int* n, int U) {
    select();
    require_weights();
    std::vector<int64_t> off(U);
    for (int u = 0; u < U; ++u) {
        if (n[u] < 0 || (int64_t)n[u] > stride) throw std::runtime_error("each utterance must hold 0..stride samples");
        off[u] = (int64_t)u * stride;
    }
    tm_.h2d_ms = 0.0;
    run_mel_utts(pcm_dev, off, n, U);
}

void Engine::upload_windows(const int* utt, const int* seek, int E) {
    if (E < 1 || E > max_batch_) throw std::runtime_error("encoder windows must be 1..max_batch");
    if (un_.empty()) throw std::runtime_error("encode_windows before load_utterances");
    whost_.assign((size_t)2 * E, 0);
    for (int e = 0; e < E; ++e) {
        if (utt[e] < 0 || utt[e] >= (int)un_.size()) throw std::runtime_error("window of an unknown utterance");
        // whisper_full only encodes at seek < n_len_org <= n / 160 + 1, so the 3000 frames lie
        // inside the (n + 480000) / 160 of the utterance's mel
        const int n_len = (int)(((int64_t)un_[utt[e]] + 480000) / 160);
        if (seek[e] < 0 || seek[e] + 3000 > n_len) throw std::runtime_error("window past the end of its utterance");
        whost_[e] = utt[e];
        whost_[E + e] = seek[e];
    }
    HIP_CHECK(hipMemcpyAsync(win_utt_, whost_.data(), (size_t)E * 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(win_seek_, whost_.data() + E, (size_t)E * 4, hipMemcpyHostToDevice, st_));
}

void Engine::encode_windows(const int* utt, const int* seek, int E) {
    select();
    require_weights();
    upload_windows(utt, seek, E);
    HIP_CHECK(hipEventRecord(ev_[2], st_));
    mel_norm(dt_, umel_, umax_, mu_, win_utt_, win_seek_, E, dm_.n_mels, cp_, mel_in_, nullptr, st_);
    HIP_CHECK(hipEventRecord(ev_[3], st_));
    enqueue_encoder(E);
    HIP_CHECK(hipEventRecord(ev_[4], st_));
    run_cross_kv(E);
    HIP_CHECK(hipEventRecord(ev_[5], st_));
    enc_E_ = E;
    enc_pending_ = true;
    cs_.encoder_windows += E;
}

// One encoder layer over the Bg windows starting at row r0 (whisper_build_graph_encoder's block:
// LN1 -> q/k/v -> attention -> out-proj + residual -> LN2 -> fc1 + GELU -> fc2 + residual).
// probe: 4 / 5 -> events e0 / e1 around fc1 / the attention (spt_probe_kernel).
void Engine::enc_layer(int l, int Bg, int64_t r0, hipStream_t s, int probe, hipEvent_t e0, hipEvent_t e1) {
    const int d = dm_.d, T = dm_.n_audio_ctx, H = dm_.n_head, M = Bg * T;
    const EncL& e = enc_[l];
    auto rows = [&](void* base, int64_t ld, int es) { return (void*)((char*)base + r0 * ld * es); };
    float* x = (float*)rows(x_, d, 4);
    void* xn = rows(xn_, d, esz_);
    void* qkv = rows(qkv_, 3 * d, esz_);
    void* ao = rows(ao_, d, esz_);
    void* ff = rows(ff_, 4 * d, esz_);
    GemmArgs g{};
    layernorm(dt_, x, M, d, e.ln1_w, e.ln1_b, xn, s);
    g.A = xn; g.lda = d; g.W = e.qkv_w; g.ldw = d; g.M = M; g.N = 3 * d; g.K = d; g.bias = e.qkv_b;
    g.C = qkv; g.ldc = 3 * d;
    g.groups = enc_groups_cur_;
    gemm_nt(dt_, EPI_BIAS, g, 1, s);
    if (probe == 5) HIP_CHECK(hipEventRecord(e0, s));
    enc_attention(dt_, qkv, Bg, T, H, ao, s);
    if (probe == 5) HIP_CHECK(hipEventRecord(e1, s));
    g = GemmArgs{};
    g.A = ao; g.lda = d; g.W = e.o_w; g.ldw = d; g.M = M; g.N = d; g.K = d; g.bias = e.o_b;
    g.C = x; g.ldc = d;
    g.groups = enc_groups_cur_;
    gemm_nt(dt_, EPI_BIAS_RESID, g, 1, s);
    layernorm(dt_, x, M, d, e.ln2_w, e.ln2_b, xn, s);
    g = GemmArgs{};
    g.A = xn; g.lda = d; g.W = e.fc1_w; g.ldw = d; g.M = M; g.N = 4 * d; g.K = d; g.bias = e.fc1_b;
    g.C = ff; g.ldc = 4 * d;
    if (probe == 4) HIP_CHECK(hipEventRecord(e0, s));
    g.groups = enc_groups_cur_;
    gemm_nt(dt_, EPI_BIAS_GELU, g, 1, s);
    if (probe == 4) HIP_CHECK(hipEventRecord(e1, s));
    g = GemmArgs{};
    g.A = ff; g.lda = 4 * d; g.W = e.fc2_w; g.ldw = 4 * d; g.M = M; g.N = d; g.K = 4 * d; g.bias = e.fc2_b;
    g.C = x; g.ldc = d;
    g.groups = enc_groups_cur_;
    gemm_nt(dt_, EPI_BIAS_RESID, g, 1, s);
}

void Engine::run_encoder(int B) {
    const int d = dm_.d, T = dm_.n_audio_ctx;
    GemmArgs g{};
    // conv1 (k3, s1, p1) + GELU -> y1p rows 1..3000
    g.A = mel_in_; g.lda = cp_; g.sA = (int64_t)MEL_ROWS * cp_;
    g.W = conv1_w_; g.ldw = 3 * cp_;
    g.M = 2 * T; g.N = d; g.K = 3 * cp_;
    g.bias = conv1_b_;
    g.C = (char*)y1p_ + (size_t)d * esz_; g.ldc = d; g.sC = (int64_t)MEL_ROWS * d;
    gemm_nt(dt_, EPI_BIAS_GELU, g, B, st_);
    // conv2 (k3, s2, p1) + GELU + positional embedding -> residual stream x (f32)
    g = GemmArgs{};
    g.A = y1p_; g.lda = 2 * d; g.sA = (int64_t)MEL_ROWS * d;
    g.W = conv2_w_; g.ldw = 3 * d;
    g.M = T; g.N = d; g.K = 3 * d;
    g.bias = conv2_b_;
    g.C = x_; g.ldc = d; g.sC = (int64_t)T * d;
    g.pos = enc_pos_;
    gemm_nt(dt_, EPI_BIAS_GELU_POS, g, B, st_);
    // The layers run per window group, each group's rows (whole windows: every kernel below is
    // row-local or per window) on its own stream, so one group's kernels fill the CUs the other's
    // leave idle: a 256 x 256-tile GEMM's last partial round, the attention's tail, the
    // memory-bound LayerNorms beside MFMA-bound GEMMs.  Every output row is computed by the same
    // operations in the same order whatever the grouping (the GEMM tile variants are bitwise
    // equal), so the grouping never changes a bit (test_encoder_groups_bitwise).
    const int G = enc_groups(B);
    int b0[kEncGroupsMax + 1];
    for (int i = 0; i <= G; ++i) b0[i] = (int)((int64_t)B * i / G);
    auto stream_of = [&](int i) { return i == 0 ? st_ : enc_st_[i - 1]; };
    if (G > 1) {
        HIP_CHECK(hipEventRecord(enc_ev_[0], st_));
        for (int i = 1; i < G; ++i) HIP_CHECK(hipStreamWaitEvent(stream_of(i), enc_ev_[0], 0));
    }
    auto rows = [&](void* base, int64_t row, int64_t ld, int es) { return (char*)base + row * ld * es; };
    enc_groups_cur_ = G;  // the layers' GEMMs of the G groups run side by side (tile choice)
    for (int l = 0; l < dm_.n_enc; ++l)
        for (int i = 0; i < G; ++i)  // layer l of every group before layer l + 1 of any
            enc_layer(l, b0[i + 1] - b0[i], (int64_t)b0[i] * T, stream_of(i));
    for (int i = 0; i < G; ++i) {
        const int64_t r0 = (int64_t)b0[i] * T;
        layernorm(dt_, (float*)rows(x_, r0, d, 4), (b0[i + 1] - b0[i]) * T, d, lnp_w_, lnp_b_,
                  rows(enc_out_, r0, d, esz_), stream_of(i));
    }
    for (int i = 1; i < G; ++i) {
        HIP_CHECK(hipEventRecord(enc_ev_[i], stream_of(i)));
        HIP_CHECK(hipStreamWaitEvent(st_, enc_ev_[i], 0));
    }
}

// Window groups of an encoder call: SPT_ENC_GROUPS (1..4, read per call; at most one group per
// window); default two groups from eight windows up (C3: groups of 6000 rows keep the 256 x 256
// tiles; r5 A/B, profiles/r5/exp_enc_groups.txt: encoder 20.15 -> 20.04 ms), else one.  Three or
// four groups at B = 8 drop the N = 1280 GEMMs to 128-row tiles and were 15-35 % slower.
int Engine::enc_groups(int B) const {
    int G = B >= 8 ? 2 : 1;
    if (const char* v = getenv("SPT_ENC_GROUPS")) G = atoi(v);
    return std::max(1, std::min({G, kEncGroupsMax, B}));
}

// The encoder is one fixed chain of launches per batch size (about 7 per layer, 230 for
// large-v3): from the second call with a given B it replays a captured graph, which removes the
// eager launch gaps between its kernels.  The first call runs eagerly, which also sets the
// kernels' one-time attributes outside any capture.  SPT_NO_GRAPH / SPT_ENC_GRAPH=0: eager.
void Engine::enqueue_encoder(int B) {
    static const bool eager = getenv("SPT_NO_GRAPH") || (getenv("SPT_ENC_GRAPH") && atoi(getenv("SPT_ENC_GRAPH")) == 0);
    const std::pair<int, int> key{B, enc_groups(B)};
    if (eager || !enc_seen_.count(key)) {
        enc_seen_.insert(key);
        run_encoder(B);
        return;
    }
    auto it = enc_graphs_.find(key);
    if (it == enc_graphs_.end()) {
        hipGraph_t graph;
        HIP_CHECK(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal));
        try {
            run_encoder(B);
        } catch (...) {
            (void)hipStreamEndCapture(st_, &graph);
            throw;
        }
        HIP_CHECK(hipStreamEndCapture(st_, &graph));
        hipGraphExec_t exec;
        HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        HIP_CHECK(hipGraphDestroy(graph));
        it = enc_graphs_.emplace(key, exec).first;
    }
    HIP_CHECK(hipGraphLaunch(it->second, st_));
}

void Engine::run_cross_kv(int B) {
    const int d = dm_.d, T = dm_.n_audio_ctx;
    GemmArgs g{};
    g.A = enc_out_; g.lda = d; g.W = ckv_w_; g.ldw = d; g.M = B * T; g.N = dm_.n_dec * 2 * d; g.K = d;
    g.bias = ckv_b_; g.C = ckv_; g.kv_B = B; g.kv_T = T; g.kv_H = dm_.n_head;
    gemm_nt(dt_, EPI_KVSPLIT, g, 1, st_);
}

// One decoder pass: 8 launches per layer.  The residual stream is f32 rows; fc2 splits K over
// 2 workgroups and leaves its result as pending partial slabs, which the next QKV LayerNorm
// prologue sums (x + slabs, fixed order) and writes to the other x buffer: no read-modify-write
// of the residual there and 2x the workgroups on the N = d projection (r1 ubench: fc2 10.2 ->
// 5.7 us).  The self- and cross-attention output projections keep the read-modify-write
// residual add: every workgroup of the LayerNorm GEMV after them re-reads the residual rows,
// so slabs there cost more than they save (cross-out: +1.2 us per slab on fc1; self-out:
// r1 exp24, in place +0.4 % RTFx over 2 slabs).
void Engine::enqueue_decoder_pass(DecGroup& g, int E, int Tq, const DecodeRequest& rq, int out_cap) {
    float* x = enqueue_layers(g, E, Tq);
    enqueue_head(g, Tq, rq, out_cap, x, suppress_, (rq.flags & 1u) != 0);
}

// The decoder layers over this pass's Tq input rows per sequence (embedded in g.dx); returns
// the residual buffer holding the result (plus g.pend's pending slabs, n = fc2's split).
float* Engine::enqueue_layers(DecGroup& g, int E, int Tq) {
    const int d = dm_.d, H = dm_.n_head, ctx = dm_.n_text_ctx, T = dm_.n_audio_ctx, B = g.B, R = B * Tq;
    const int64_t self_layer = (int64_t)2 * B * H * ctx * 64, cross_layer = kv_layer_elems(E, H, T);
    // window map: rows j * share .. + share - 1 attend to window g.kvrow[j * share]; without one,
    // row b attends to window g.b0 + b (the cross-attention key split applies there only)
    const bool mapped = g.share > 0;
    const int runs = B / std::max(1, g.share);
    // a small grid (B = 1: 20 workgroups; a beam's 5 rows on one window: 20) streams each window's
    // K/V through few CUs: run its 8 waves as 8 workgroups, merged in the output projection, and
    // for one-token steps of shared rows one query per workgroup (the 8 x 5 workgroups per head
    // re-read the window's 384 KB from L2) -- all bitwise the same result.  r4
    // (profiles/r4/exp_xattn_vw.txt, exp_beam_step.txt): B = 1 pass 1.609 -> 1.562 ms; the 5-query
    // workgroups of a beam took 29 us per layer; B = 8 (160 workgroups) stays on the 8-wave kernel.
    // SPT_XATTN_VW=0: never, 2: always, 3: small grids without the per-query split (measurements and
    // the cross-strategy bitwise tests; read when a pass is captured, so a new engine picks it up)
    const int vw_env = getenv("SPT_XATTN_VW") ? atoi(getenv("SPT_XATTN_VW")) : 1;
    const bool vw = vw_env == 2 || (vw_env != 0 && runs * H < 96);
    const bool per_query = vw && Tq == 1 && vw_env != 3;
    // the 8 partials merged by the cross output projection's prologue for one row (B = 1: cheaper
    // than a launch), by a merge kernel for more (the prologue repeats the merge in each of its
    // 80 workgroups: 15 us at a beam's 5 rows)
    const bool vw_merge = vw && R > 1;
    const int xs = vw ? (vw_merge ? 1 : 8) : mapped ? 1 : xsplit_;
    const int ks = dt_ == DT_BF16 ? 128 : 64;
    hipStream_t st = g.st;
    float* xc = g.dx;   // current residual rows (dec_embed / dec_finalize wrote this pass's input here)
    float* xo = g.dx2;  // the other buffer
    int np = 0;         // pending slabs in g.pend
    pend_fold_ = !getenv("SPT_DEC_XFOLD") || atoi(getenv("SPT_DEC_XFOLD")) != 0;
    auto ln_input = [&](GemvArgs& a) {  // LayerNorm prologue over xc + the pending slabs
        ln_source(a, xc, g.pend, np, (int64_t)R * d);
        a.x_out = np > 0 ? xo : nullptr;
    };
    auto consumed = [&] {
        if (np > 0) std::swap(xc, xo);
        np = 0;
    };
    // probe(): events around the probed kernel of every layer (eager passes only)
    auto pmark = [&](int kind, int l, int which) {
        if (probe_kind_ == kind) HIP_CHECK(hipEventRecord(probe_ev_[2 * l + which], st));
    };
    auto partial = [&](GemvArgs& a, int split) {  // a K-split projection producing pending slabs
        a.C = g.pend; a.ldc = d; a.c_split = (int64_t)R * d;
        a.ksplit = split;
        a.p_resid = pend_fold_ ? xc : nullptr;
        if (a.K / ks < split) throw std::runtime_error("decoder projection too narrow for its K split");
        np = split;
    };
    for (int l = 0; l < dm_.n_dec; ++l) {
        const DecL& e = dec_[l];
        void* skv_l = (char*)g.skv + self_layer * l * esz_;
        // layer l of the cross K/V (kv_offset layout, E windows), at this group's first window when
        // the rows map to windows one to one
        const void* ckv_l = (const char*)ckv_ + (cross_layer * l + (mapped ? 0 : (int64_t)g.b0 * H * 4096)) * esz_;
        // LN1 + QKV projection + self K/V append, then the self-attention
        {
            GemvArgs a{};
            ln_input(a); a.lda = d; a.ln_w = e.ln1_w; a.ln_b = e.ln1_b; a.R = R;
            a.W = e.qkv_w; a.N = 3 * d; a.K = d; a.bias = e.qkv_b; a.C = g.dq; a.ldc = d;
            a.cache = skv_l; a.cache_B = B; a.cache_H = H; a.cache_ctx = ctx; a.Tq = Tq; a.st = g.ds;
            gemv(dt_, GV_QKV_CACHE, A_LN, a, st);
            consumed();
            pmark(1, l, 0);
            dec_self_attn(dt_, g.dq, skv_l, B, H, ctx, Tq, g.ds, g.dao, st);
            pmark(1, l, 1);
        }
        // self-attention output projection, residual add in place: the cross-Q LayerNorm
        // prologue then reads x alone (r1 exp24: +0.4 % RTFx over a 2-way K split into slabs)
        GemvArgs a{};
        a.A = g.dao; a.lda = d; a.R = R; a.W = e.so_w; a.N = d; a.K = d; a.bias = e.so_b;
        a.C = xc; a.ldc = d;
        gemv(dt_, GV_BIAS_RESID, A_DIRECT, a, st);
        // LN2 + cross-Q projection
        a = GemvArgs{};
        ln_input(a); a.lda = d; a.ln_w = e.ln2_w; a.ln_b = e.ln2_b; a.R = R;
        a.W = e.cq_w; a.N = d; a.K = d; a.bias = e.cq_b; a.C = g.dq; a.ldc = d;
        gemv(dt_, GV_BIAS, A_LN, a, st);
        consumed();
        pmark(0, l, 0);
        if (vw)
        {
            dec_cross_attn_vw(dt_, g.dq, ckv_l, B, E, H, T, Tq, g.xpart, st, mapped ? g.kvrow : nullptr,
                              mapped ? g.share : 1, per_query);
            if (vw_merge) dec_attn_part_merge(dt_, g.xpart, R, H, g.dao, st);
        }
        else
            dec_cross_attn(dt_, g.dq, ckv_l, B, E, H, T, Tq, g.dao, st, xs, g.xpart, mapped ? g.kvrow : nullptr,
                           mapped ? g.share : 1);
        pmark(0, l, 1);
        // cross output projection (merging the key chunks in its prologue), residual add in place
        a = GemvArgs{};
        a.A = g.dao; a.lda = d; a.R = R; a.W = e.co_w; a.N = d; a.K = d; a.bias = e.co_b; a.C = xc; a.ldc = d;
        if (xs > 1) { a.apart = g.xpart; a.a_splits = xs; a.a_heads = H; }
        gemv(dt_, GV_BIAS_RESID, xs > 1 ? A_ATTN : A_DIRECT, a, st);
        // LN3 + fc1 + GELU
        a = GemvArgs{};
        ln_input(a); a.lda = d; a.ln_w = e.ln3_w; a.ln_b = e.ln3_b; a.R = R;
        a.W = e.fc1_w; a.N = 4 * d; a.K = d; a.bias = e.fc1_b; a.C = g.dff; a.ldc = 4 * d;
        pmark(3, l, 0);
        gemv(dt_, GV_BIAS_GELU, A_LN, a, st);
        pmark(3, l, 1);
        consumed();
        // fc2 -> pending slabs
        a = GemvArgs{};
        a.A = g.dff; a.lda = 4 * d; a.R = R; a.W = e.fc2_w; a.N = d; a.K = 4 * d; a.bias = e.fc2_b;
        partial(a, fc2_split_);
        gemv(dt_, GV_PARTIAL, A_DIRECT, a, st);
    }
    return xc;
}

void Engine::ln_source(GemvArgs& a, float* xc, float* pend, int np, int64_t slab) const {
    // x + p0 + p1 + ...; with the residual folded into slab 0 the sum starts at slab 0 (the same
    // additions in the same order: bitwise the same rows)
    const int f = np > 0 && pend_fold_ ? 1 : 0;
    a.A = f ? pend : xc;
    for (int p = 0; p < kMaxPend; ++p) a.pend[p] = p < np - f ? pend + (int64_t)(p + f) * slab : zero_;
    a.n_pend = np - f;
}

// Final LayerNorm of each sequence's last row + logits (suppression mask `sup`, the step-0
// blank rule when `blank`) + top-2 partials, then argmax / record / next embedding / advance.
void Engine::enqueue_head(DecGroup& g, int Tq, const DecodeRequest& rq, int out_cap, float* xc,
                          const uint32_t* sup, bool blank) {
    const int d = dm_.d, ctx = dm_.n_text_ctx, B = g.B, R = B * Tq;
    hipStream_t st = g.st;
    const Specials sp = specials_for(dm_.n_vocab);
    const int n_tiles = (dm_.n_vocab + 15) / 16;
    GemvArgs a{};
    // final LayerNorm of the last token of each sequence (x + fc2's pending slabs); the
    // combined rows are not needed
    ln_source(a, xc, g.pend, fc2_split_, (int64_t)R * d);
    a.lda = Tq * d; a.a_row0 = (Tq - 1) * d; a.ln_w = lnf_w_; a.ln_b = lnf_b_; a.R = B;
    a.W = tok_emb_; a.N = dm_.n_vocab; a.K = d; a.C = g.logits; a.ldc = dm_.n_vocab; a.st = g.ds;
    a.suppress = sup;
    a.blank0 = blank ? sp.eot : -1;
    a.blank1 = blank ? 220 : -1;
    a.part = g.part; a.n_tiles = n_tiles;
    gemv(dt_, GV_LOGITS, A_LN, a, st);
    if (rq.beam_k > 0) {  // candidates for the host's beam bookkeeping; no token is chosen here
        BeamArgs bm{};
        bm.logits = g.logits; bm.ldl = dm_.n_vocab;
        bm.n_vocab = dm_.n_vocab; bm.eot = sp.eot; bm.beg = sp.beg; bm.blank = rq.blank_tok;
        bm.suppress = sup; bm.prm = g.prm; bm.row = g.beam_row; bm.step = g.beam_step; bm.k = rq.beam_k;
        bm.cand_id = g.cand_id; bm.cand_lp = g.cand_lp; bm.tid = g.beam_tid;
        static const bool one_wg = getenv("SPT_BEAM_ONE_WG") != nullptr;  // the single-workgroup kernel (A/B)
        bm.stat = one_wg ? nullptr : g.beam_stat;
        dec_beam_topk(bm, B, st);
        dec_advance(g.ds, Tq, st);
        return;
    }
    if (rq.full) {
        TsArgs t{};
        t.logits = g.logits; t.ldl = dm_.n_vocab;
        t.n_vocab = dm_.n_vocab; t.eot = sp.eot; t.beg = sp.beg; t.blank = rq.blank_tok;
        t.suppress = sup; t.prm = g.prm; t.seek = g.seek; t.seek_end = g.seek_end; t.state = g.ts_state;
        t.forced = rq.n_forced > 0 ? g.forced : nullptr; t.forced_len = rq.n_forced;
        t.next_tok = g.tok_in; t.out_tok = g.out_tok; t.out_plog = g.out_t1; t.out_tid = g.out_t2; t.out_cap = out_cap;
        t.done = g.done;
        t.emb = tok_emb_; t.pos = dec_pos_; t.d = d; t.ctx = ctx; t.Tq = Tq; t.x = g.dx;
        t.ds = g.ds; t.arrive = g.arrive; t.stat = g.ts_stat;
        dec_ts_stats(t, B, st);
        dec_finalize_ts(dt_, t, B, st);
        return;
    }
    FinalizeArgs f{};
    f.part = g.part; f.n_tiles = n_tiles;
    f.eot = sp.eot; f.ignore_eot = (rq.flags & 4u) ? 1 : 0; f.n_vocab = dm_.n_vocab;
    f.forced = rq.n_forced > 0 ? g.forced : nullptr; f.forced_len = rq.n_forced;
    f.next_tok = g.tok_in; f.out_tok = g.out_tok; f.out_top1 = g.out_t1; f.out_top2 = g.out_t2; f.out_cap = out_cap;
    f.done = g.done;
    f.emb = tok_emb_; f.pos = dec_pos_; f.d = d; f.ctx = ctx; f.Tq = Tq; f.x = g.dx;
    f.ds = g.ds; f.arrive = g.arrive;
    dec_finalize(dt_, f, B, st);
}

void Engine::run_decode(int B, const DecodeRequest& rq, int* tokens, float* top1, float* top2, int* lang_out,
                        int* ts_state_out) {
    const int Tq = (int)rq.prompt.size();
    const int ctx = dm_.n_text_ctx;
    const int P = rq.row_prefix.empty() ? (int)rq.prefix.size() : (int)rq.row_prefix[0].size();
    if (Tq < 1 || Tq > 4) throw std::runtime_error("prompt must have 1..4 tokens");
    if (B < 1 || B > max_batch_) throw std::runtime_error("batch out of range");
    const int E = enc_E_;
    if (E < 1) throw std::runtime_error("decode before encode_windows");
    // the rows' window map: S = rows per window (consecutive runs of equal length), 0 = none
    int S = 0;
    if (!rq.kv_row.empty()) {
        if ((int)rq.kv_row.size() != B) throw std::runtime_error("kv_row needs one window per row");
        for (int v : rq.kv_row)
            if (v < 0 || v >= E) throw std::runtime_error("kv_row names a window that was not encoded");
        S = 1;
        for (int sh = std::min(8, B); sh > 1 && S == 1; --sh) {
            if (B % sh) continue;
            bool ok = true;
            for (int b = 0; b < B && ok; ++b) ok = rq.kv_row[b] == rq.kv_row[b - b % sh];
            if (ok) S = sh;
        }
    } else if (B > E) {
        throw std::runtime_error("more decoder rows than encoded windows (and no kv_row map)");
    }
    // decoder passes carry at most max_rows_ rows: a batch above that is split over decode
    // groups (in whole windows of S rows), and a group whose prompt rows exceed it prefills the
    // prompt a chunk of tokens at a time (the same rows, positions and keys) and runs the logits
    // pass on the last prompt token alone
    auto group_split = [&](int unit_rows, int* G_out) {  // -> the largest group's rows
        const int nU = B / unit_rows;
        *G_out = std::min((int)groups_.size(),
                          std::max(std::min(n_groups_, nU), cdiv(nU, std::max(1, max_rows_ / unit_rows))));
        return cdiv(nU, *G_out) * unit_rows;
    };
    int G = 0;
    int Bg = group_split(std::max(1, S), &G);
    // whole windows of S rows do not always fit the groups (groups_ is sized for rows split at any
    // point: e.g. f32 medium, 23 rows per pass, 3 groups at max_batch 64: best_of 6 over 10 windows
    // puts 4 windows = 24 rows in the largest group); the window
    // map then runs with one row per run (share 1), which every strategy computes bitwise the same
    if (S > 1 && Bg > max_rows_) {
        S = 1;
        Bg = group_split(1, &G);
    }
    const int unit = std::max(1, S), nU = B / unit;
    if (Bg > max_rows_) throw std::runtime_error("batch exceeds the decoder's rows per pass");
    const int cmax = std::max(1, std::min(4, max_rows_ / Bg));
    const int Tq_head = Bg * Tq > max_rows_ ? 1 : Tq;
    if (P > ctx / 2 + 1) throw std::runtime_error("prompt prefix longer than n_text_ctx / 2 + 1");
    for (int t : rq.prefix)
        if (t < 0 || t >= dm_.n_vocab) throw std::runtime_error("prompt token out of the vocabulary");
    if (!rq.lang_tok.empty() && ((int)rq.lang_tok.size() != B || Tq < 3))
        throw std::runtime_error("per-sequence language tokens need a [sot, lang, task, ...] prompt");
    if (rq.n_steps < 1 || P + Tq + rq.n_steps > ctx + 1) throw std::runtime_error("n_steps out of range");
    if (rq.n_forced > ctx) throw std::runtime_error("too many forced tokens");
    const int out_cap = rq.n_steps;
    const Specials sp = specials_for(dm_.n_vocab);
    // always-suppressed ids (whisper_process_logits); the fast path also masks the timestamps
    // here, the whisper_full path applies its timestamp rules per step (k_sample.hip)
    const uint32_t sflags = (rq.flags & 2u) | (rq.full ? 0x100u : 0u);
    if (suppress_flags_ != sflags || suppress_extra_ != rq.extra_suppress) {
        const int V = dm_.n_vocab;
        host_suppress_.assign(V / 32 + 1, 0u);
        auto set = [&](int i) { if (i >= 0 && i < V) host_suppress_[i >> 5] |= 1u << (i & 31); };
        set(sp.not_);
        if ((rq.flags & 2u) && !rq.full)
            for (int i = sp.beg; i < V; ++i) set(i);
        set(sp.sot); set(sp.nosp); set(sp.solm); set(sp.translate); set(sp.transcribe); set(sp.prev);
        for (int i = 0; i < sp.n_langs; ++i) set(sp.sot + 1 + i);
        for (int i : rq.extra_suppress) set(i);
        HIP_CHECK(hipMemcpyAsync(suppress_, host_suppress_.data(), host_suppress_.size() * 4, hipMemcpyHostToDevice, st_));
        HIP_CHECK(hipStreamSynchronize(st_));
        suppress_flags_ = sflags;
        suppress_extra_ = rq.extra_suppress;
    }
    if (rq.full && ((int)rq.seek.size() != B || (int)rq.seek_end.size() != B))
        throw std::runtime_error("whisper_full decoding needs seek / seek_end per sequence");
    if (!rq.row_prefix.empty()) {
        if ((int)rq.row_prefix.size() != B) throw std::runtime_error("row_prefix needs one prefix per sequence");
        for (const auto& r : rq.row_prefix) {
            if (r.size() != rq.row_prefix[0].size()) throw std::runtime_error("row prefixes must have equal lengths");
            for (int t : r)
                if (t < 0 || t >= dm_.n_vocab) throw std::runtime_error("prompt token out of the vocabulary");
        }
    }
    // split the batch over the decode groups; each waits for the encoder / cross-K/V
    HIP_CHECK(hipEventRecord(ev_[6], st_));
    std::vector<DecGroup*> act;
    kvrow_host_ = rq.kv_row;  // host source of the asynchronous uploads below
    for (int gi = 0, b0 = 0; gi < G; ++gi) {
        DecGroup& g = groups_[gi];
        g.b0 = b0;
        g.B = (nU / G + (gi < nU % G ? 1 : 0)) * unit;
        g.share = S;
        b0 += g.B;
        act.push_back(&g);
        HIP_CHECK(hipStreamWaitEvent(g.st, ev_[6], 0));
        if (S > 0)
            HIP_CHECK(hipMemcpyAsync(g.kvrow, kvrow_host_.data() + g.b0, (size_t)g.B * 4, hipMemcpyHostToDevice, g.st));
        // host sources of this call's token uploads (kept alive in the group until the next call)
        g.host_tok.assign((size_t)g.B * (P + Tq + 8), 0);
        g.host_used = 0;
        if (rq.n_forced > 0)
            HIP_CHECK(hipMemcpyAsync(g.forced, rq.forced + (size_t)g.b0 * rq.n_forced, (size_t)g.B * rq.n_forced * 4,
                                     hipMemcpyHostToDevice, g.st));
        if (rq.full) {  // pageable sources: copied before the call returns
            HIP_CHECK(hipMemcpyAsync(g.seek, rq.seek.data() + g.b0, g.B * 4, hipMemcpyHostToDevice, g.st));
            HIP_CHECK(hipMemcpyAsync(g.seek_end, rq.seek_end.data() + g.b0, g.B * 4, hipMemcpyHostToDevice, g.st));
            HIP_CHECK(hipMemcpyAsync(g.prm, &rq.ts, sizeof(TsParams), hipMemcpyHostToDevice, g.st));
        }
    }
    auto upload_tokens = [&](DecGroup& g, const std::function<int(int, int)>& tok, int n) {  // [g.B][n]
        int* h = g.host_tok.data() + g.host_used;
        for (int b = 0; b < g.B; ++b)
            for (int t = 0; t < n; ++t) h[b * n + t] = tok(g.b0 + b, t);
        g.host_used += g.B * n;
        HIP_CHECK(hipMemcpyAsync(g.tok_in, h, (size_t)g.B * n * 4, hipMemcpyHostToDevice, g.st));
    };
    ts_init_.clear();  // a member: the source of asynchronous copies outlives this function
    for (int b = 0; b < B; ++b) ts_init_.insert(ts_init_.end(), {0, 3000, 0, 0});
    auto reset_outputs = [&](DecGroup& g) {
        HIP_CHECK(hipMemsetAsync(g.done, 0, g.B * 4, g.st));
        HIP_CHECK(hipMemsetAsync(g.out_tok, 0xFF, (size_t)g.B * out_cap * 4, g.st));
        fill_f32(g.out_t1, (int64_t)g.B * out_cap, -INFINITY, g.st);
        fill_f32(g.out_t2, (int64_t)g.B * out_cap, -INFINITY, g.st);
        dec_reset(g.ds, g.arrive, g.st);
        if (rq.full)  // WHISPER_DECODER_INIT: seek_delta starts at a whole window (3000 frames)
            HIP_CHECK(hipMemcpyAsync(g.ts_state, ts_init_.data() + (size_t)g.b0 * 4, g.B * 16, hipMemcpyHostToDevice,
                                     g.st));
    };
    // language auto-detection (whisper_lang_auto_detect_with_state): one pass on [sot] with every
    // non-language token suppressed; the argmax is the language token
    std::vector<int> lang(B, -1);
    bool detect = false;
    for (int v : rq.lang_tok) detect = detect || v < 0;
    if (detect) {
        if (sp.n_langs <= 0) throw std::runtime_error("language detection needs a multilingual model");
        if (!suppress_lang_ready_) {
            const int V = dm_.n_vocab;
            std::vector<uint32_t> m(V / 32 + 1, ~0u);
            for (int i = 0; i < sp.n_langs; ++i) m[(sp.sot + 1 + i) >> 5] &= ~(1u << ((sp.sot + 1 + i) & 31));
            HIP_CHECK(hipMemcpy(suppress_lang_, m.data(), m.size() * 4, hipMemcpyHostToDevice));
            suppress_lang_ready_ = true;
        }
        DecodeRequest dq;  // no forcing, no blank rule, EOT irrelevant; the fast head
        dq.flags = 4u;
        for (DecGroup* g : act) {
            reset_outputs(*g);
            upload_tokens(*g, [&](int, int) { return sp.sot; }, 1);
            dec_embed(dt_, g->tok_in, g->B, 1, dm_.d, tok_emb_, dec_pos_, g->ds, g->dx, g->st);
            float* x = enqueue_layers(*g, E, 1);
            enqueue_head(*g, 1, dq, out_cap, x, suppress_lang_, false);
        }
        std::vector<int> first((size_t)B * out_cap);
        for (DecGroup* g : act) {
            HIP_CHECK(hipMemcpyAsync(first.data() + (size_t)g->b0 * out_cap, g->out_tok, (size_t)g->B * out_cap * 4,
                                     hipMemcpyDeviceToHost, g->st));
            HIP_CHECK(hipStreamSynchronize(g->st));
        }
        for (int b = 0; b < B; ++b) {
            const int v = rq.lang_tok[b];
            lang[b] = v >= 0 ? v : first[(size_t)(-v - 1) * out_cap];
            if (lang[b] <= sp.sot || lang[b] > sp.sot + sp.n_langs) throw std::runtime_error("language detection failed");
        }
    } else if (!rq.lang_tok.empty()) {
        for (int b = 0; b < B; ++b) lang[b] = rq.lang_tok[b];
    }
    if (lang_out)
        for (int b = 0; b < B; ++b) lang_out[b] = lang[b] >= 0 ? lang[b] : (Tq >= 3 ? rq.prompt[1] : -1);
    for (DecGroup* gp : act) {
        DecGroup& g = *gp;
        reset_outputs(g);
        // whisper_full prompt_past ([prev] + prompt tokens): prefilled in chunks of <= 4 rows per
        // sequence through the decoder layers only (no logits), positions 0..P-1
        const bool rows = !rq.row_prefix.empty();
        const int P = rows ? (int)rq.row_prefix[0].size() : (int)rq.prefix.size();
        for (int c0 = 0; c0 < P; c0 += cmax) {
            const int n = std::min(cmax, P - c0);
            upload_tokens(g, [&](int b, int t) { return rows ? rq.row_prefix[b][c0 + t] : rq.prefix[c0 + t]; }, n);
            dec_embed(dt_, g.tok_in, g.B * n, n, dm_.d, tok_emb_, dec_pos_, g.ds, g.dx, g.st);
            enqueue_layers(g, E, n);
            dec_advance(g.ds, n, g.st);
        }
        auto prompt_tok = [&](int b, int t) { return (t == 1 && lang[b] >= 0) ? lang[b] : rq.prompt[t]; };
        for (int c0 = 0; c0 < Tq - Tq_head; c0 += cmax) {  // only when Bg * Tq > max_rows_
            const int n = std::min(cmax, Tq - Tq_head - c0);
            upload_tokens(g, [&](int b, int t) { return prompt_tok(b, c0 + t); }, n);
            dec_embed(dt_, g.tok_in, g.B * n, n, dm_.d, tok_emb_, dec_pos_, g.ds, g.dx, g.st);
            enqueue_layers(g, E, n);
            dec_advance(g.ds, n, g.st);
        }
        upload_tokens(g, [&](int b, int t) { return prompt_tok(b, Tq - Tq_head + t); }, Tq_head);
        dec_embed(dt_, g.tok_in, g.B * Tq_head, Tq_head, dm_.d, tok_emb_, dec_pos_, g.ds, g.dx, g.st);
        if (rq.beam_k > 0) {  // the first step's state: no tokens yet
            beam_host_.assign((size_t)g.B * 4 + 1, 0);
            for (int b = 0; b < g.B; ++b) beam_host_[b * 4 + 3] = 3000;
            HIP_CHECK(hipMemcpyAsync(g.beam_row, beam_host_.data(), (size_t)g.B * 16, hipMemcpyHostToDevice, g.st));
            HIP_CHECK(hipMemcpyAsync(g.beam_step, beam_host_.data() + (size_t)g.B * 4, 4, hipMemcpyHostToDevice, g.st));
        }
        enqueue_decoder_pass(g, E, Tq_head, rq, out_cap);  // prompt pass produces token 0
    }
    if (rq.beam_k > 0) {  // beam search continues step by step from the host (beam_next)
        tm_.n_decode_passes = 1;
        for (DecGroup* g : act) {
            HIP_CHECK(hipEventRecord(g->ev, g->st));
            HIP_CHECK(hipStreamWaitEvent(st_, g->ev, 0));
        }
        return;
    }
    int passes = 1;
    static const bool no_graph = getenv("SPT_NO_GRAPH") != nullptr;  // eager passes (profilers, debugging)
    static const bool sync_debug = getenv("SPT_DEBUG_SYNC") != nullptr;  // per-pass sync + state check
    if (rq.n_steps > 1 && no_graph) {
        for (int s = 1; s < rq.n_steps; ++s, ++passes)
            for (DecGroup* g : act) {
                enqueue_decoder_pass(*g, E, 1, rq, out_cap);
                if (!sync_debug) continue;
                const hipError_t e = hipStreamSynchronize(g->st);
                DecState h{};
                if (e == hipSuccess) HIP_CHECK(hipMemcpy(&h, g->ds, sizeof(h), hipMemcpyDeviceToHost));
                if (e != hipSuccess || h.step != s + 1 || (s % 16) == 0)
                    fprintf(stderr, "[spt] pass %d: %s step=%d pos0=%d\n", s, hipGetErrorString(e), h.step, h.pos0);
                if (e != hipSuccess) throw HipError(std::string("pass failed: ") + hipGetErrorString(e));
            }
    } else if (rq.n_steps > 1) {
        std::vector<hipGraphExec_t> ex;
        for (DecGroup* g : act) {
            // E and b0 are baked into the captured cross-K/V addresses, the window map's share
            // into the cross-attention grid (the map itself is read from g->kvrow)
            GraphKey key{g->B, E, g->b0, out_cap, rq.n_forced, rq.flags, rq.full};
            key.share = S;
            auto it = g->graphs.find(key);
            if (it == g->graphs.end()) {
                hipGraph_t graph;
                HIP_CHECK(hipStreamBeginCapture(g->st, hipStreamCaptureModeThreadLocal));
                enqueue_decoder_pass(*g, E, 1, rq, out_cap);
                HIP_CHECK(hipStreamEndCapture(g->st, &graph));
                hipGraphExec_t exec;
                HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
                HIP_CHECK(hipGraphDestroy(graph));
                it = g->graphs.emplace(key, exec).first;
            }
            ex.push_back(it->second);
        }
        const bool early_exit = !(rq.flags & 4u);
        std::vector<int> hdone(B);
        for (int s = 1; s < rq.n_steps; ++s) {
            for (size_t i = 0; i < act.size(); ++i) HIP_CHECK(hipGraphLaunch(ex[i], act[i]->st));
            ++passes;
            if (early_exit && (s % 16) == 0) {
                bool all = true;
                for (DecGroup* g : act) {
                    HIP_CHECK(hipMemcpyAsync(hdone.data(), g->done, g->B * 4, hipMemcpyDeviceToHost, g->st));
                    HIP_CHECK(hipStreamSynchronize(g->st));
                    all = all && std::all_of(hdone.begin(), hdone.begin() + g->B, [](int v) { return v != 0; });
                }
                if (all) break;
            }
        }
    }
    tm_.n_decode_passes = passes;
    for (DecGroup* g : act) {
        const size_t off = (size_t)g->b0 * out_cap, n = (size_t)g->B * out_cap * 4;
        HIP_CHECK(hipMemcpyAsync(tokens + off, g->out_tok, n, hipMemcpyDeviceToHost, g->st));
        if (top1) HIP_CHECK(hipMemcpyAsync(top1 + off, g->out_t1, n, hipMemcpyDeviceToHost, g->st));
        if (top2) HIP_CHECK(hipMemcpyAsync(top2 + off, g->out_t2, n, hipMemcpyDeviceToHost, g->st));
        if (ts_state_out && rq.full)
            HIP_CHECK(hipMemcpyAsync(ts_state_out + (size_t)g->b0 * 4, g->ts_state, (size_t)g->B * 16,
                                     hipMemcpyDeviceToHost, g->st));
        HIP_CHECK(hipEventRecord(g->ev, g->st));
        HIP_CHECK(hipStreamWaitEvent(st_, g->ev, 0));
    }
}

void Engine::decode(int B, const DecodeRequest& rq, int* tokens, float* top1, float* top2, int* lang_out,
                    int* ts_state_out) {
    select();
    require_weights();
    HIP_CHECK(hipEventRecord(ev_[6], st_));  // the decode groups wait for the encoded windows here
    run_decode(B, rq, tokens, top1, top2, lang_out, ts_state_out);
    HIP_CHECK(hipEventRecord(ev_[7], st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    HIP_CHECK(hipGetLastError());
    tm_.batch = B;
    cs_.engine_calls++;
    cs_.decoder_passes += tm_.n_decode_passes;
    finish_call_timing();
}

// phase times of the stages since the last decode (HIP events; read after its synchronisation)
void Engine::finish_call_timing() {
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[6], ev_[7]));
    tm_.decode_ms = ms;
    double total = ms;
    if (enc_pending_) {
        float m_norm, m_enc, m_kv;
        HIP_CHECK(hipEventElapsedTime(&m_norm, ev_[2], ev_[3]));
        HIP_CHECK(hipEventElapsedTime(&m_enc, ev_[3], ev_[4]));
        HIP_CHECK(hipEventElapsedTime(&m_kv, ev_[4], ev_[5]));
        tm_.encoder_ms = m_enc;
        tm_.cross_kv_ms = m_kv;
        tm_.mel_ms = m_norm;
        cs_.encoder_ms += m_enc;
        total += m_norm + m_enc + m_kv;
    } else {
        tm_.encoder_ms = tm_.cross_kv_ms = tm_.mel_ms = 0.0;
    }
    if (mel_pending_) {
        HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
        tm_.mel_ms += ms;
        total += ms;
    }
    // the sum of the stage intervals: host work between the stages (whisper_full's bookkeeping
    // between load_utterances, encode_windows and decode) is not device time
    tm_.total_ms = total;
    cs_.device_ms += total;
    cs_.decode_ms += tm_.decode_ms;
    mel_pending_ = enc_pending_ = false;
}

void Engine::transcribe_device(const float* pcm_dev, int64_t stride, const int* n_samples, int B,
                               const DecodeRequest& rq, int* tokens, float* top1, float* top2, int* lang_out,
                               int* ts_state_out) {
    if (B < 1 || B > max_batch_) throw std::runtime_error("batch exceeds the context's max_batch");
    for (int b = 0; b < B; ++b)
        if (n_samples[b] < 0 || n_samples[b] > 480000 || (int64_t)n_samples[b] > stride)
            throw std::runtime_error("each window must hold 0..480000 samples within its stride");
    load_utterances_device(pcm_dev, stride, n_samples, B);
    std::vector<int> utt(B), seek(B, 0);
    for (int b = 0; b < B; ++b) utt[b] = b;
    encode_windows(utt.data(), seek.data(), B);
    decode(B, rq, tokens, top1, top2, lang_out, ts_state_out);
}

void Engine::transcribe_host(const float* const* pcm, const int* n_samples, int B, const DecodeRequest& rq,
                             int* tokens, float* top1, float* top2, int* lang_out, int* ts_state_out) {
    if (B < 1 || B > max_batch_) throw std::runtime_error("batch exceeds the context's max_batch");
    for (int b = 0; b < B; ++b)
        if (n_samples[b] < 0 || n_samples[b] > 480000) throw std::runtime_error("window longer than 30 s");
    load_utterances(pcm, n_samples, B);
    std::vector<int> utt(B), seek(B, 0);
    for (int b = 0; b < B; ++b) utt[b] = b;
    encode_windows(utt.data(), seek.data(), B);
    decode(B, rq, tokens, top1, top2, lang_out, ts_state_out);
}

// ----------------------------------------------------------------------------- beam search
void Engine::read_cands(int B, BeamCands* out) {
    DecGroup& g = groups_[0];
    out->id.resize((size_t)B * 8);
    out->lp.resize((size_t)B * 8);
    out->tid.resize(B);
    // cand_id, cand_lp and beam_tid are consecutive carvings of one workspace: one copy back
    const char* lo = (const char*)g.cand_id;
    const size_t o_lp = (const char*)g.cand_lp - lo, o_tid = (const char*)g.beam_tid - lo;
    beam_rd_.resize(o_tid + (size_t)B * 4);
    HIP_CHECK(hipMemcpyAsync(beam_rd_.data(), lo, beam_rd_.size(), hipMemcpyDeviceToHost, g.st));
    HIP_CHECK(hipStreamSynchronize(g.st));
    memcpy(out->id.data(), beam_rd_.data(), (size_t)B * 32);
    memcpy(out->lp.data(), beam_rd_.data() + o_lp, (size_t)B * 32);
    memcpy(out->tid.data(), beam_rd_.data() + o_tid, (size_t)B * 4);
}

void Engine::beam_begin(int B, const DecodeRequest& rq, BeamCands* out, int* lang_out) {
    select();
    require_weights();
    if (rq.beam_k < 1 || rq.beam_k > 8) throw std::runtime_error("beam size must be in 1..8");
    if (n_groups_ != 1) throw std::runtime_error("beam search needs one decode group");
    if (B > max_rows_)
        throw std::runtime_error("beam search rows (utterances x beam_size) exceed the decoder's " +
                                 std::to_string(max_rows_) + " rows per pass for this model");
    if (!kvtmp_) {
        const size_t bytes = (size_t)dm_.n_dec * 2 * max_batch_ * dm_.n_head * dm_.n_text_ctx * 64 * esz_;
        if (hipMalloc(&kvtmp_, bytes) != hipSuccess) {
            kvtmp_ = nullptr;
            throw std::runtime_error("out of device memory for the beam search scratch");
        }
        // finite from the start: the self-attention reads a wave's first key block before it knows
        // the position (rows past it are masked, p = 0, and must not hold NaN / Inf bit patterns)
        HIP_CHECK(hipMemset(kvtmp_, 0, bytes));
    }
    beam_rq_ = rq;
    beam_B_ = B;
    beam_side_ = 0;  // the prompt pass writes the group's own cache
    std::vector<int> tok((size_t)B * rq.n_steps);
    decode(B, rq, tok.data(), nullptr, nullptr, lang_out, nullptr);
    read_cands(B, out);
}

void Engine::beam_next(const int* src, const int* tokens, const int* rowstate, int step, BeamCands* out) {
    select();
    const int B = beam_B_;
    if (B < 1) throw std::runtime_error("beam_next without beam_begin");
    DecGroup& g = groups_[0];
    for (int b = 0; b < B; ++b)
        if (src[b] < 0 || src[b] >= B || tokens[b] < 0 || tokens[b] >= dm_.n_vocab)
            throw std::runtime_error("beam_next: bad source row or token");
    // host sources stay alive until the step's results are read back (synchronous below).  beam_row,
    // beam_step and beam_src are consecutive carvings of one workspace: one upload for the three,
    // laid out at their device offsets, and one for the tokens
    char* lo = (char*)g.beam_row;
    const size_t o_step = (char*)g.beam_step - lo, o_src = (char*)g.beam_src - lo;
    beam_host_.assign((o_src + (size_t)B * 4 + 3) / 4, 0);
    char* hb = (char*)beam_host_.data();
    memcpy(hb, rowstate, (size_t)B * 16);
    memcpy(hb + o_step, &step, 4);
    memcpy(hb + o_src, src, (size_t)B * 4);
    beam_tok_.assign(tokens, tokens + B);
    HIP_CHECK(hipMemcpyAsync(lo, hb, o_src + (size_t)B * 4, hipMemcpyHostToDevice, g.st));
    HIP_CHECK(hipMemcpyAsync(g.tok_in, beam_tok_.data(), (size_t)B * 4, hipMemcpyHostToDevice, g.st));
    // one captured graph per (rows, candidates, flags, length, cache side): gather the self-K/V
    // rows (positions < pos0) from the side holding them into the other side, which this step's
    // layers then append to and read (the two sides alternate: one gather per step, not a gather
    // into the scratch and a copy back), feed the tokens, the decoder pass and the candidates
    // kernel.  The uploads above stay outside: the graph reads them in place.  (The next window's
    // prompt pass writes the group's own cache from position 0, so either side may end a search.)
    const int side = beam_side_;
    void* const own = g.skv;
    void* const kv_from = side ? kvtmp_ : own;
    void* const kv_to = side ? own : kvtmp_;
    auto beam_pass = [&] {
        dec_kv_gather(dt_, kv_from, kv_to, g.beam_src, dm_.n_dec, B, dm_.n_head, dm_.n_text_ctx, g.ds, g.st);
        dec_embed(dt_, g.tok_in, B, 1, dm_.d, tok_emb_, dec_pos_, g.ds, g.dx, g.st);
        struct SkvSide {  // the layers append to / read kv_to; the group's pointer is restored on unwind
            DecGroup& g;
            void* own;
            ~SkvSide() { g.skv = own; }
        } side_guard{g, own};
        g.skv = kv_to;
        float* x = enqueue_layers(g, enc_E_, 1);
        g.skv = own;
        enqueue_head(g, 1, beam_rq_, beam_rq_.n_steps, x, suppress_, (beam_rq_.flags & 1u) != 0);
    };
    static const bool no_graph = getenv("SPT_NO_GRAPH") != nullptr;
    HIP_CHECK(hipEventRecord(ev_[8], g.st));
    if (no_graph) {
        beam_pass();
    } else {
        // n_forced = -beam_k marks a beam-step graph (a real n_forced is >= 0)
        GraphKey key{B, enc_E_, side, beam_rq_.n_steps, -beam_rq_.beam_k, beam_rq_.flags, beam_rq_.full};  // b0: cache side
        key.share = g.share;
        auto it = g.graphs.find(key);
        if (it == g.graphs.end()) {
            hipGraph_t graph;
            HIP_CHECK(hipStreamBeginCapture(g.st, hipStreamCaptureModeThreadLocal));
            beam_pass();
            HIP_CHECK(hipStreamEndCapture(g.st, &graph));
            hipGraphExec_t exec;
            HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
            HIP_CHECK(hipGraphDestroy(graph));
            it = g.graphs.emplace(key, exec).first;
        }
        HIP_CHECK(hipGraphLaunch(it->second, g.st));
    }
    HIP_CHECK(hipEventRecord(ev_[9], g.st));
    read_cands(B, out);  // synchronises g.st
    beam_side_ ^= 1;
    float ms = 0.0f;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[8], ev_[9]));
    cs_.beam_steps++;
    cs_.decoder_passes++;
    cs_.device_ms += ms;
    cs_.decode_ms += ms;
}

// ----------------------------------------------------------------------------- debug hooks
void Engine::debug_mel(const float* pcm_host, int n, int seek, float* out_host) {
    select();
    const float* p = pcm_host;
    load_utterances(&p, &n, 1);
    const int u = 0;
    upload_windows(&u, &seek, 1);
    mel_pending_ = false;
    float* dbg = nullptr;
    const size_t bytes = (size_t)dm_.n_mels * 3000 * 4;
    HIP_CHECK(hipMalloc(&dbg, bytes));
    mel_norm(dt_, umel_, umax_, mu_, win_utt_, win_seek_, 1, dm_.n_mels, cp_, mel_in_, dbg, st_);
    HIP_CHECK(hipMemcpyAsync(out_host, dbg, bytes, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    HIP_CHECK(hipFree(dbg));
}

void Engine::debug_encode(const float* mel_host, float* out_host) {
    select();
    require_weights();
    const int nm = dm_.n_mels, d = dm_.d, T = dm_.n_audio_ctx;
    std::vector<char> img((size_t)MEL_ROWS * cp_ * esz_, 0);
    for (int t = 0; t < 3000; ++t)
        for (int c = 0; c < nm; ++c) {
            const float v = mel_host[(size_t)c * 3000 + t];
            const size_t o = (size_t)(t + 1) * cp_ + c;
            if (esz_ == 2) ((uint16_t*)img.data())[o] = f2bf(v);
            else ((float*)img.data())[o] = v;
        }
    HIP_CHECK(hipMemcpyAsync(mel_in_, img.data(), img.size(), hipMemcpyHostToDevice, st_));
    run_encoder(1);
    float* tmp = nullptr;
    HIP_CHECK(hipMalloc(&tmp, (size_t)T * d * 4));
    to_f32(dt_, enc_out_, tmp, (int64_t)T * d, st_);
    HIP_CHECK(hipMemcpyAsync(out_host, tmp, (size_t)T * d * 4, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    HIP_CHECK(hipFree(tmp));
}

bool Engine::debug_weight_checksum(int tid, double* out2) {
    select();
    auto it = tref_.find(tid);
    if (it == tref_.end()) return false;
    HIP_CHECK(hipMemsetAsync(scratch_, 0, 16, st_));
    tensor_checksum(it->second.dt, it->second.p, it->second.n, scratch_, st_);
    HIP_CHECK(hipMemcpyAsync(out2, scratch_, 16, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    return true;
}

}  // namespace spt

namespace spt {

double Engine::probe(int kind, int iters, double* work, int* is_flops) {
    select();
    const int B = enc_E_;  // the encoded windows (cross K/V layout, encoder batch)
    if (B < 1 || tm_.batch < 1) throw std::runtime_error("probe needs a completed transcription call first");
    if (iters < 1 || iters > 100000) throw std::runtime_error("iters out of range");
    const int d = dm_.d, H = dm_.n_head, T = dm_.n_audio_ctx, ctx = dm_.n_text_ctx, V = dm_.n_vocab;
    DecGroup& g = groups_[0];
    const int Bg = g.B > 0 ? g.B : B;
    // kinds 0 and 3 launch the kernel of nl different decoder layers back to back (as in the
    // decode loop: each on its own, cache-cold weights / K/V); the time is per launch
    const int nl = (kind == 0 || kind == 3) ? std::min(8, dm_.n_dec) : 1;
    std::function<void()> launch;
    *is_flops = 0;
    switch (kind) {
        case 0:  // cross-attention of layers 0..nl-1 (one launch each) over this group's cross K/V
            launch = [&] {
                for (int l = 0; l < nl; ++l)
                    dec_cross_attn(dt_, g.dq, (const char*)ckv_ + kv_layer_elems(B, H, T) * l * esz_, std::min(Bg, B), B,
                                   H, T, 1, g.dao, st_, xsplit_, g.xpart);
            };
            *work = 2.0 * std::min(Bg, B) * H * T * 64 * esz_;
            break;
        case 1:
            launch = [&] { dec_self_attn(dt_, g.dq, g.skv, Bg, H, ctx, 1, g.ds, g.dao, st_); };
            {
                DecState h{};
                HIP_CHECK(hipMemcpy(&h, g.ds, sizeof(h), hipMemcpyDeviceToHost));
                *work = 2.0 * Bg * H * (h.pos0 + 1) * 64 * esz_;
            }
            break;
        case 2: {
            launch = [&] {
                GemvArgs a{};
                a.A = g.dx; a.lda = d; a.ln_w = lnf_w_; a.ln_b = lnf_b_; a.R = Bg;
                for (int p = 0; p < kMaxPend; ++p) a.pend[p] = zero_;
                a.W = tok_emb_; a.N = V; a.K = d; a.C = g.logits; a.ldc = V; a.st = g.ds;
                a.suppress = suppress_; a.blank0 = a.blank1 = -1; a.part = g.part; a.n_tiles = (V + 15) / 16;
                gemv(dt_, GV_LOGITS, A_LN, a, st_);
            };
            *work = (double)V * d * esz_;
            break;
        }
        case 3: {
            launch = [&] {
                GemvArgs a{};
                for (int l = 0; l < nl; ++l) {
                    a.A = g.dx; a.lda = d; a.ln_w = dec_[l].ln3_w; a.ln_b = dec_[l].ln3_b; a.R = Bg;
                    for (int p = 0; p < kMaxPend; ++p) a.pend[p] = zero_;
                    a.W = dec_[l].fc1_w; a.N = 4 * d; a.K = d; a.bias = dec_[l].fc1_b; a.C = g.dff; a.ldc = 4 * d;
                    gemv(dt_, GV_BIAS_GELU, A_LN, a, st_);
                }
            };
            *work = 4.0 * d * d * esz_;
            break;
        }
        case 4: {
                    launch = [&] {
                GemmArgs a{};
                a.A = xn_; a.lda = d; a.W = enc_[0].fc1_w; a.ldw = d; a.M = B * T; a.N = 4 * d; a.K = d;
                a.bias = enc_[0].fc1_b; a.C = ff_; a.ldc = 4 * d;
                gemm_nt(dt_, EPI_BIAS_GELU, a, 1, st_);
            };
            *work = 2.0 * B * T * 4.0 * d * d;
            *is_flops = 1;
            break;
        }
        case 5:
            launch = [&] { enc_attention(dt_, qkv_, B, T, H, ao_, st_); };
            *work = 4.0 * B * H * (double)T * T * 64;
            *is_flops = 1;
            break;
        default:
            throw std::runtime_error("unknown probe kind");
    }
    if (n_groups_ > 1 || dm_.n_enc < 1) {
        if (kind >= 4 && dm_.n_enc < 1) throw std::runtime_error("model has no encoder layers");
    }
    launch();  // warm
    static const bool insitu = getenv("SPT_PROBE_INSITU") && atoi(getenv("SPT_PROBE_INSITU")) != 0;
    if (kind <= 3 && insitu) {
        // decoder kernels in situ (SPT_PROBE_INSITU=1): eager one-token passes over the last call's
        // rows, with events around the probed kernel of every layer (cross-attention,
        // self-attention, fc1) or around the logits launch after the layers.  Each pair also holds
        // the launch's dispatch and completion latency: r5 read the cross-attention 2.7 us (19 %)
        // above its rocprofv3 average this way, so the default stays the back-to-back timing
        // below (r4: within 1 % for the cross-attention).  The layers rewrite the self-K/V row of
        // the current position with the same values, and the head is not run, so no sequence
        // state moves.
        const int L = dm_.n_dec;
        if ((int)probe_ev_.size() < 2 * L) {
            for (int i = (int)probe_ev_.size(); i < 2 * L; ++i) {
                hipEvent_t e;
                HIP_CHECK(hipEventCreate(&e));
                probe_ev_.push_back(e);
            }
        }
        HIP_CHECK(hipStreamSynchronize(st_));  // the warm-up launch
        const int passes = std::max(1, iters / (kind == 2 ? 1 : L));
        double tot = 0.0;
        int n = 0;
        for (int i = 0; i < passes; ++i) {
            probe_kind_ = kind == 2 ? -1 : kind;
            float* x = nullptr;
            try {
                x = enqueue_layers(g, enc_E_, 1);
            } catch (...) {
                probe_kind_ = -1;
                throw;
            }
            probe_kind_ = -1;
            if (kind == 2) {
                GemvArgs a{};
                ln_source(a, x, g.pend, fc2_split_, (int64_t)Bg * d);
                a.lda = d; a.ln_w = lnf_w_; a.ln_b = lnf_b_; a.R = Bg;
                a.W = tok_emb_; a.N = V; a.K = d; a.C = g.logits; a.ldc = V; a.st = g.ds;
                a.suppress = suppress_; a.blank0 = a.blank1 = -1; a.part = g.part; a.n_tiles = (V + 15) / 16;
                HIP_CHECK(hipEventRecord(probe_ev_[0], g.st));
                gemv(dt_, GV_LOGITS, A_LN, a, g.st);
                HIP_CHECK(hipEventRecord(probe_ev_[1], g.st));
            }
            HIP_CHECK(hipStreamSynchronize(g.st));
            for (int l = 0; l < (kind == 2 ? 1 : L); ++l) {
                float ms;
                HIP_CHECK(hipEventElapsedTime(&ms, probe_ev_[2 * l], probe_ev_[2 * l + 1]));
                tot += ms;
                ++n;
            }
        }
        return tot * 1000.0 / n;
    }
    if (kind <= 3) {
        // decoder kernels: inside the decode loop their operands come from HBM (a pass streams
        // ~4 GB through the 256 MB Infinity Cache), so each timed group of launches follows a
        // read of 512 MB of other weights, and only the launches are between the two events
        const int64_t fb = std::min<int64_t>(wbytes_, (int64_t)512 << 20) & ~(int64_t)15;
        double tot = 0.0;
        iters = std::max(1, iters / nl);
        for (int i = 0; i < iters; ++i) {
            cache_flush(warena_, fb, (unsigned*)scratch_, st_);
            HIP_CHECK(hipEventRecord(ev_[0], st_));
            launch();
            HIP_CHECK(hipEventRecord(ev_[1], st_));
            HIP_CHECK(hipEventSynchronize(ev_[1]));
            float ms;
            HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
            tot += ms;
        }
        return tot * 1000.0 / (iters * nl);
    }
    if (kind == 4 || kind == 5) {
        // encoder kernels inside the encoder's own sequence: `iters` back-to-back runs of encoder
        // layer 0's launches on the last call's buffers (enc_layer: LN1, q/k/v, attention, out, LN2,
        // fc1, fc2), with an event pair around the probed kernel of each run and one host wait at the
        // end, so the kernel follows its producer, on a chip as busy (and as hot)
        // as inside the encoder.  r4's back-to-back repeats of the kernel alone read the attention
        // 10 % below its rocprofv3 average, r5's producer-then-kernel pairs with a host wait
        // between them 8 % below.  The residual rows x grow by one layer per run: the probe runs
        // after the timed calls, and every call recomputes them.
        if ((int)probe_ev_.size() < 2 * iters) {
            for (int i = (int)probe_ev_.size(); i < 2 * iters; ++i) {
                hipEvent_t ev;
                HIP_CHECK(hipEventCreate(&ev));
                probe_ev_.push_back(ev);
            }
        }
        enc_groups_cur_ = 1;  // one full-batch launch per kernel
        for (int i = 0; i < iters; ++i) enc_layer(0, B, 0, st_, kind, probe_ev_[2 * i], probe_ev_[2 * i + 1]);
        HIP_CHECK(hipStreamSynchronize(st_));
        double tot = 0.0;
        for (int i = 0; i < iters; ++i) {
            float ms;
            HIP_CHECK(hipEventElapsedTime(&ms, probe_ev_[2 * i], probe_ev_[2 * i + 1]));
            tot += ms;
        }
        return tot * 1000.0 / iters;
    }
    HIP_CHECK(hipEventRecord(ev_[0], st_));
    for (int i = 0; i < iters; ++i) launch();
    HIP_CHECK(hipEventRecord(ev_[1], st_));
    HIP_CHECK(hipEventSynchronize(ev_[1]));
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
    return ms * 1000.0 / iters;
}

}  // namespace spt
