// parakeet.cpp -- Parakeet-V3 engine: weights, workspace and the per-call launch sequence.
//
// Reference path: TranscriptionManager loads ParakeetEngine with ParakeetModelParams::int8()
// (/root/reference/src-tauri/src/managers/transcription.rs:278-297) and calls
// transcribe_samples(audio, Some(ParakeetInferenceParams { timestamp_granularity: Segment }))
// (transcription.rs:505-513); transcribe-rs 0.2.3 runs the parakeet-tdt-0.6b-v3 ONNX export
// through ONNX Runtime.  Here the same model (NeMo FastConformer-TDT, oracle/parakeet_oracle.h)
// runs as: GPU log-mel (DFT as an f32 MFMA GEMM), dw_striding subsampling, 24 Conformer layers
// (fp16 MFMA GEMMs with fused bias / Swish / ReLU / scaled-residual epilogues), and TDT greedy
// decoding on the device with all utterances of the batch stepping together in a hipGraph.
#include "parakeet.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

constexpr int kMaxSymbols = 16;  // max_symbols bound (the output capacity per frame)
constexpr int kStepsPerGraph = 8;

int fanin_exp(int K) { return (int)floor(log2(sqrt(3.0 / (double)K)) + 0.5); }
int round_up(int x, int m) { return (x + m - 1) / m * m; }
int halve(int t) { return (t - 1) / 2 + 1; }
// a stride-2 conv stage's valid length (0 stays 0)
int sub_len(int t) { return t > 0 ? halve(t) : 0; }

struct Carve {
    char* base;
    int64_t off = 0;
    void* take(int64_t bytes) {
        off = (off + 255) & ~(int64_t)255;
        void* p = base ? base + off : nullptr;
        off += bytes;
        return p;
    }
};

// librosa-style slaney mel filterbank, exactly as oracle/po_model.c computes it (f64 -> f32)
void slaney_filters(int n_mels, std::vector<float>* fb) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
    auto hz2mel = [&](double f) { return f < min_log_hz ? f / f_sp : min_log_mel + log(f / min_log_hz) / logstep; };
    auto mel2hz = [&](double z) { return z < min_log_mel ? f_sp * z : min_log_hz * exp(logstep * (z - min_log_mel)); };
    const double mlo = hz2mel(0.0), mhi = hz2mel(8000.0);
    std::vector<double> pts(n_mels + 2);
    for (int i = 0; i < n_mels + 2; i++) pts[i] = mel2hz(mlo + (mhi - mlo) * i / (n_mels + 1));
    fb->assign((size_t)n_mels * PK_NBIN, 0.0f);
    for (int j = 0; j < n_mels; j++) {
        const double en = 2.0 / (pts[j + 2] - pts[j]);
        for (int k = 0; k < PK_NBIN; k++) {
            const double fk = 8000.0 * k / 256.0;
            const double lo = (fk - pts[j]) / (pts[j + 1] - pts[j]), hi = (pts[j + 2] - fk) / (pts[j + 2] - pts[j + 1]);
            const double v = lo < hi ? lo : hi;
            (*fb)[(size_t)j * PK_NBIN + k] = (float)((v > 0 ? v : 0.0) * en);
        }
    }
}

}  // namespace

bool parse_parakeet_spec(const std::string& spec, PkDims* dm, uint64_t* seed, std::string* err) {
    const std::string pre = "synthetic:";
    if (spec.compare(0, pre.size(), pre) != 0) return false;
    std::vector<std::string> parts;
    size_t s = pre.size();
    while (true) {
        const size_t e = spec.find(':', s);
        parts.push_back(spec.substr(s, e == std::string::npos ? std::string::npos : e - s));
        if (e == std::string::npos) break;
        s = e + 1;
    }
    PkDims d;
    d.name = parts[0];
    if (d.name == "parakeet-tdt-0.6b-v3") {
        // defaults
    } else if (d.name == "parakeet-tdt-0.6b-v2") {
        // the catalog's English-only model (model_catalog.json:214-217): v3's network with a
        // 1024-piece SentencePiece vocabulary [upstream, recalled]
        d.n_vocab = 1024;
    } else if (d.name == "parakeet-test-small") {
        d.d = 256; d.n_layers = 2; d.n_heads = 4; d.ff = 1024; d.sub_ch = 128; d.pred = 128; d.n_vocab = 1024;
    } else {
        *err = "unknown synthetic Parakeet model '" + d.name + "'";
        return true;
    }
    for (size_t i = 1; i < parts.size(); ++i) {
        const std::string& p = parts[i];
        const size_t eq = p.find('=');
        if (eq == std::string::npos) { *err = "bad spec option '" + p + "'"; return true; }
        const std::string k = p.substr(0, eq), v = p.substr(eq + 1);
        char* end = nullptr;
        const unsigned long long x = strtoull(v.c_str(), &end, 10);
        if (v.empty() || *end) { *err = "bad value in '" + p + "'"; return true; }
        if (k == "layers" && x >= 1 && x <= 64) d.n_layers = (int)x;
        else if (k == "seed") *seed = x;
        else { *err = "unknown or out-of-range spec option '" + p + "'"; return true; }
    }
    *dm = d;
    return true;
}

void ParakeetEngine::select() const { HIP_CHECK(hipSetDevice(dev_)); }

ParakeetEngine::ParakeetEngine(const PkDims& dm, int dtype, int device, int max_batch, int max_samples, uint64_t seed,
                               bool synthetic_weights)
    : dm_(dm), dt_(dtype), dev_(device), max_batch_(max_batch), max_samples_(max_samples), seed_(seed) {
    if (max_batch < 1 || max_batch > 64) throw std::runtime_error("max_batch must be in [1, 64]");
    if (max_samples < 1600 || max_samples > 16000 * 1200) throw std::runtime_error("max_samples must be in [0.1 s, 20 min]");
    if (dm_.d % dm_.n_heads || (dm_.d / dm_.n_heads) % 8) throw std::runtime_error("head dim must be a multiple of 8");
    if (dm_.pred % 128 || dm_.d % 256 || dm_.ff % 256 || dm_.sub_ch % 128)
        throw std::runtime_error("Parakeet dims must be multiples of the GEMM tiles (pred % 128, d % 256, ff % 256, sub_ch % 128)");
    esz_ = dtype == DT_F32 ? 4 : 2;
    F1_ = halve(dm_.n_mels);
    F2_ = halve(F1_);
    F3_ = halve(F2_);
    set_frame_limits();
    const int P = dm_.pred;
    P_pad_ = round_up(P, 64);
    joint_pad_ = round_up(dm_.n_vocab + 1 + dm_.n_dur, 64);
    joint_tiles_ = joint_pad_ / pk_joint_tile();
    select();
    try {
        HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
        ev_.resize(6);
        for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
        pk_prepare();
        gemm_prepare();
        alloc_weights();
        alloc_workspace();
        upload_tables();
        if (synthetic_weights) {
            for (const TSpec& t : specs_) {
                gen_weights(DT_F32, scratch_, t.n, seed_, (uint32_t)t.tid, t.kind, t.exp, st_);
                SPT_LAUNCH_CHECK();
                place(t, scratch_);
            }
            HIP_CHECK(hipStreamSynchronize(st_));
        }
    } catch (...) {
        release();
        throw;
    }
}

ParakeetEngine::~ParakeetEngine() { release(); }

void ParakeetEngine::release() {
    (void)hipSetDevice(dev_);
    if (st_) (void)hipStreamSynchronize(st_);
    for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
    graphs_.clear();
    for (auto& kv : enc_graphs_) (void)hipGraphExecDestroy(kv.second);
    enc_graphs_.clear();
    for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
    for (auto& e : prof_ev_) if (e) (void)hipEventDestroy(e);
    ev_.clear();
    prof_ev_.clear();
    if (warena_) (void)hipFree(warena_);
    if (aarena_) (void)hipFree(aarena_);
    if (scratch_) (void)hipFree(scratch_);
    if (win_) (void)hipFree(win_);
    if (basis_) (void)hipFree(basis_);
    if (fbT_) (void)hipFree(fbT_);
    if (pin_) (void)hipHostFree(pin_);
    pin_ = nullptr;
    pin_cap_ = 0;
    if (hst_pin_) (void)hipHostFree(hst_pin_);
    hst_pin_ = nullptr;
    hst_cap_ = 0;
    if (res_pin_) (void)hipHostFree(res_pin_);
    res_pin_ = nullptr;
    res_cap_ = 0;
    warena_ = aarena_ = nullptr;
    scratch_ = win_ = basis_ = fbT_ = nullptr;
    if (st_) (void)hipStreamDestroy(st_);
    st_ = nullptr;
}

// Tensor table: ids, generator scales and kinds exactly as oracle/po_model.c build_table; each
// tensor is placed into its engine layout (GEMM weights [N][K] in the storage dtype; the
// prediction network / joint W^T [K][Npad] f32 for the lanes-over-outputs GEMVs; q / k / v
// stacked; every layer's linear_pos stacked for one GEMM; the subsampling output weight's
// columns permuted from (channel, freq) to the engine's channel-last (freq, channel) flatten)
void ParakeetEngine::alloc_weights() {
    const int C = dm_.sub_ch, d = dm_.d, K = dm_.conv_k, P = dm_.pred, V1 = dm_.n_vocab + 1;
    const int NO = V1 + dm_.n_dur, ff = dm_.ff, Ln = dm_.n_layers;
    const int64_t dd = (int64_t)d * d;
    const int PLAIN = WK_MAT, PLUS1 = WK_LNW;
    for (int pass = 0; pass < 2; ++pass) {
        Carve c{warena_};
        specs_.clear();
        auto F32 = [&](int64_t n) { return (float*)c.take(n * 4); };
        auto TT = [&](int64_t n) { return c.take(n * esz_); };
        auto add = [&](int tid, int64_t n, int kind, int exp, int mode, int dt, void* dst, int N = 1, int Kd = 0,
                       int ld = 0, int row0 = 0) {
            specs_.push_back(TSpec{tid, n, kind, exp, mode, dt, dst, N, Kd ? Kd : (int)n, ld, row0});
        };
        auto f32t = [&](int tid, int64_t n, int kind, int exp) {
            float* p = F32(n);
            add(tid, n, kind, exp, PK_PLACE_COPY, DT_F32, p);
            return p;
        };
        auto mat = [&](int tid, int64_t n, int fan, void* dst) { add(tid, n, PLAIN, fanin_exp(fan), PK_PLACE_COPY, dt_, dst); };
        c0_w_ = f32t(1, (int64_t)C * 9, PLAIN, fanin_exp(9));
        c0_b_ = f32t(2, C, PLAIN, -5);
        dw1_w_ = f32t(3, (int64_t)C * 9, PLAIN, fanin_exp(9));
        dw1_b_ = f32t(4, C, PLAIN, -5);
        pw1_w_ = TT((int64_t)C * C); mat(5, (int64_t)C * C, C, pw1_w_);
        pw1_b_ = f32t(6, C, PLAIN, -5);
        dw2_w_ = f32t(7, (int64_t)C * 9, PLAIN, fanin_exp(9));
        dw2_b_ = f32t(8, C, PLAIN, -5);
        pw2_w_ = TT((int64_t)C * C); mat(9, (int64_t)C * C, C, pw2_w_);
        pw2_b_ = f32t(10, C, PLAIN, -5);
        sub_w_ = TT((int64_t)d * C * F3_);
        add(11, (int64_t)d * C * F3_, PLAIN, fanin_exp(C * F3_), PK_PLACE_SUBPERM, dt_, sub_w_, d, C * F3_, C, F3_);
        sub_b_ = f32t(12, d, PLAIN, -5);
        pos_w_ = TT((int64_t)Ln * dd);
        L_.assign(Ln, Layer{});
        for (int l = 0; l < Ln; ++l) {
            Layer& y = L_[l];
            const int b = 1000 + 64 * l;
            y.ln1_w = f32t(b + 0, d, PLUS1, -3);
            y.ln1_b = f32t(b + 1, d, PLAIN, -4);
            y.ff1_w1 = TT((int64_t)ff * d); mat(b + 2, (int64_t)ff * d, d, y.ff1_w1);
            y.ff1_b1 = f32t(b + 3, ff, PLAIN, -5);
            y.ff1_w2 = TT((int64_t)ff * d); mat(b + 4, (int64_t)ff * d, ff, y.ff1_w2);
            y.ff1_b2 = f32t(b + 5, d, PLAIN, -5);
            y.lna_w = f32t(b + 6, d, PLUS1, -3);
            y.lna_b = f32t(b + 7, d, PLAIN, -4);
            y.qkv_w = TT(3 * dd);
            y.qkv_b = F32(3 * d);
            for (int q = 0; q < 3; ++q) {
                mat(b + 8 + 2 * q, dd, d, (char*)y.qkv_w + q * dd * esz_);
                add(b + 9 + 2 * q, d, PLAIN, -5, PK_PLACE_COPY, DT_F32, y.qkv_b + q * d);
            }
            y.o_w = TT(dd); mat(b + 14, dd, d, y.o_w);
            y.o_b = f32t(b + 15, d, PLAIN, -5);
            mat(b + 16, dd, d, (char*)pos_w_ + l * dd * esz_);
            y.pos_u = f32t(b + 17, d, PLAIN, -4);
            y.pos_v = f32t(b + 18, d, PLAIN, -4);
            y.lnc_w = f32t(b + 19, d, PLUS1, -3);
            y.lnc_b = f32t(b + 20, d, PLAIN, -4);
            y.pw1_w = TT(2 * dd); mat(b + 21, 2 * dd, d, y.pw1_w);
            y.pw1_b = f32t(b + 22, 2 * d, PLAIN, -5);
            y.dw_w = f32t(b + 23, (int64_t)d * K, PLAIN, fanin_exp(K));
            y.dw_b = f32t(b + 24, d, PLAIN, -5);
            y.bn_g = f32t(b + 25, d, PLUS1, -3);
            y.bn_b = f32t(b + 26, d, PLAIN, -4);
            y.bn_m = f32t(b + 27, d, PLAIN, -4);
            y.bn_v = f32t(b + 28, d, PLUS1, -2);
            y.pw2_w = TT(dd); mat(b + 29, dd, d, y.pw2_w);
            y.pw2_b = f32t(b + 30, d, PLAIN, -5);
            y.ln2_w = f32t(b + 31, d, PLUS1, -3);
            y.ln2_b = f32t(b + 32, d, PLAIN, -4);
            y.ff2_w1 = TT((int64_t)ff * d); mat(b + 33, (int64_t)ff * d, d, y.ff2_w1);
            y.ff2_b1 = f32t(b + 34, ff, PLAIN, -5);
            y.ff2_w2 = TT((int64_t)ff * d); mat(b + 35, (int64_t)ff * d, ff, y.ff2_w2);
            y.ff2_b2 = f32t(b + 36, d, PLAIN, -5);
            y.lno_w = f32t(b + 37, d, PLUS1, -3);
            y.lno_b = f32t(b + 38, d, PLAIN, -4);
        }
        emb_ = f32t(90000, (int64_t)V1 * P, PLAIN, -2);
        for (int j = 0; j < 2; ++j) {
            lstm_wt_[j] = F32((int64_t)2 * P * 4 * P);
            add(90001 + 4 * j, (int64_t)4 * P * P, PLAIN, fanin_exp(P), PK_PLACE_LSTM, DT_F32, lstm_wt_[j], 4 * P, P,
                4 * P, 0);
            add(90002 + 4 * j, (int64_t)4 * P * P, PLAIN, fanin_exp(P), PK_PLACE_LSTM, DT_F32, lstm_wt_[j], 4 * P, P,
                4 * P, P);
            lstm_bih_[j] = f32t(90003 + 4 * j, 4 * P, PLAIN, -5);
            lstm_bhh_[j] = f32t(90004 + 4 * j, 4 * P, PLAIN, -5);
        }
        jenc_w_ = f32t(90009, (int64_t)P * d, PLAIN, fanin_exp(d));
        jenc_b_ = f32t(90010, P, PLAIN, -5);
        jpred_wt_ = F32((int64_t)P * P_pad_);
        add(90011, (int64_t)P * P, PLAIN, fanin_exp(P), PK_PLACE_BLOCKED, PKD_PRED, jpred_wt_, P, P, P_pad_, 0);
        jpred_b_ = F32(P_pad_);
        add(90012, P, PLAIN, -5, PK_PLACE_COPY, DT_F32, jpred_b_);
        jout_wt_ = F32((int64_t)P * joint_pad_);
        add(90013, (int64_t)NO * P, PLAIN, fanin_exp(P), PK_PLACE_BLOCKED, PKD_JOINT, jout_wt_, NO, P, joint_pad_, 0);
        jout_b_ = F32(joint_pad_);
        add(90014, NO, PLAIN, -5, PK_PLACE_COPY, DT_F32, jout_b_);
        if (!pass) {
            wbytes_ = c.off;
            if (hipMalloc(&warena_, wbytes_) != hipSuccess) {
                warena_ = nullptr;
                throw std::runtime_error("out of device memory for weights (" + std::to_string(wbytes_) + " B)");
            }
            HIP_CHECK(hipMemsetAsync(warena_, 0, wbytes_, st_));  // W^T padding, unloaded tensors
        }
    }
    table_.clear();
    int64_t mx = 0;
    for (size_t i = 0; i < specs_.size(); ++i) {
        table_[specs_[i].tid] = i;
        mx = std::max(mx, specs_[i].n);
    }
    scratch_n_ = mx;
    if (hipMalloc(&scratch_, mx * 4) != hipSuccess) {
        scratch_ = nullptr;
        throw std::runtime_error("out of device memory for the weight staging buffer");
    }
}

void ParakeetEngine::place(const TSpec& t, const float* src) {
    if (t.mode == PK_PLACE_LSTM) pk_place_lstm(src, dm_.pred, (float*)t.dst, t.row0, st_);
    else if (t.mode == PK_PLACE_BLOCKED) pk_place_blocked(src, t.N, t.K, t.dt, (float*)t.dst, st_);
    else if (t.mode == PK_PLACE_TRANSPOSE) pk_place(PK_PLACE_TRANSPOSE, DT_F32, src, t.N, t.K, t.dst, t.ld, t.row0, 0, 0, st_);
    else if (t.mode == PK_PLACE_SUBPERM) pk_place(PK_PLACE_SUBPERM, t.dt, src, t.N, 0, t.dst, 0, 0, t.ld, t.row0, st_);
    else pk_place(PK_PLACE_COPY, t.dt, src, 1, (int)t.n, t.dst, 0, 0, 0, 0, st_);
    if (t.tid == 90000)  // the prediction network's blank row is zero (blank_as_pad)
        HIP_CHECK(hipMemsetAsync((float*)t.dst + (size_t)dm_.n_vocab * dm_.pred, 0, (size_t)dm_.pred * 4, st_));
}

int64_t ParakeetEngine::tensor_numel(int tid) const {
    auto it = table_.find(tid);
    return it == table_.end() ? -1 : specs_[it->second].n;
}

void ParakeetEngine::set_tensor(int tid, const float* host, int64_t n) {
    auto it = table_.find(tid);
    if (it == table_.end()) throw std::runtime_error("unknown Parakeet tensor id " + std::to_string(tid));
    const TSpec& t = specs_[it->second];
    if (n != t.n)
        throw std::runtime_error("tensor " + std::to_string(tid) + ": " + std::to_string(n) + " elements, expected " +
                                 std::to_string(t.n));
    select();
    HIP_CHECK(hipMemcpyAsync(scratch_, host, (size_t)n * 4, hipMemcpyHostToDevice, st_));
    place(t, scratch_);
    HIP_CHECK(hipStreamSynchronize(st_));
}

void ParakeetEngine::set_frame_limits() {
    Tmax_ = max_samples_ / PK_HOP;
    T1max_ = halve(Tmax_);
    T2max_ = halve(T1max_);
    T3max_ = halve(T2max_);
    cap_ = T3max_ * kMaxSymbols + 1;
}

bool ParakeetEngine::reserve_samples(int n, int64_t max_bytes) {
    if (n <= max_samples_) return true;
    if (n > 16000 * 1200) return false;
    // grow by at least a quarter (a dictation session's recordings lengthen a little at a time),
    // in whole 80 ms encoder frames
    int64_t want = std::max<int64_t>(n, (int64_t)max_samples_ + max_samples_ / 4);
    want = std::min<int64_t>(round_up((int)std::min<int64_t>(want, 16000 * 1200), 1280), 16000 * 1200);
    // the workspace is linear in max_samples up to a few fixed-size buffers: project its size
    const double per = (double)abytes_ / max_samples_;
    if (per * want > (double)max_bytes) return false;
    select();
    HIP_CHECK(hipStreamSynchronize(st_));
    for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
    graphs_.clear();
    for (auto& kv : enc_graphs_) (void)hipGraphExecDestroy(kv.second);
    enc_graphs_.clear();
    enc_seen_.clear();
    const int old = max_samples_;
    HIP_CHECK(hipFree(aarena_));
    aarena_ = nullptr;
    // the last call's encoder output lived in the freed workspace: no completed call remains
    enc_out_ = nullptr;
    enc_out_graph_.clear();
    last_lens_.clear();
    for (int& v : last_dims_) v = 0;
    max_samples_ = (int)want;
    set_frame_limits();
    try {
        alloc_workspace();
    } catch (const std::exception&) {  // no room: back to the old size (just freed, so it fits)
        max_samples_ = old;
        set_frame_limits();
        alloc_workspace();
        return false;
    }
    HIP_CHECK(hipStreamSynchronize(st_));
    return true;
}

void ParakeetEngine::alloc_workspace() {
    const int B = max_batch_, C = dm_.sub_ch, d = dm_.d, P = dm_.pred, Ln = dm_.n_layers;
    const int64_t M3 = (int64_t)B * T3max_;
    for (int pass = 0; pass < 2; ++pass) {
        Carve c{aarena_};
        pcm_ = (float*)c.take((int64_t)B * max_samples_ * 4);
        nsamp_ = (int*)c.take(B * 4);
        lens_ = (int*)c.take(B * 16);
        frames_ = (float*)c.take((int64_t)B * Tmax_ * PK_NFFT * 4);
        spec_ = (float*)c.take((int64_t)B * Tmax_ * PK_DFT_N * 4);
        mel_ = (float*)c.take((int64_t)B * Tmax_ * dm_.n_mels * 4);
        y1_ = c.take((int64_t)B * T1max_ * F1_ * C * esz_);
        y2a_ = c.take((int64_t)B * T2max_ * F2_ * C * esz_);
        y2_ = c.take((int64_t)B * T2max_ * F2_ * C * esz_);
        y3a_ = c.take((int64_t)B * T3max_ * F3_ * C * esz_);
        y3_ = c.take((int64_t)B * T3max_ * F3_ * C * esz_);
        x_ = (float*)c.take(M3 * d * 4 * 2);  // ping-pong pair
        xn_ = c.take(M3 * d * esz_);
        ffh_ = c.take(M3 * dm_.ff * esz_);
        qkv_ = c.take(M3 * 3 * d * esz_);
        pe_ = c.take((int64_t)(2 * T3max_ - 1) * d * esz_);
        pp_ = c.take((int64_t)(2 * T3max_ - 1) * Ln * d * esz_);
        ctx_ = c.take(M3 * d * esz_);
        glu_ = c.take(M3 * 2 * d * esz_);
        cv_ = c.take(M3 * d * esz_);
        fe_ = (float*)c.take(M3 * P * 4);
        slab_ = (float*)c.take(std::max<int64_t>(M3, 32768) * d * 4);  // split-K slabs: ks * M <= ~25k rows (gemm())
        state_ = (PkState*)c.take(B * sizeof(PkState));
        h_ = (float*)c.take((int64_t)4 * B * P * 4);  // [layer][parity][B][P]
        c_ = (float*)c.take((int64_t)4 * B * P * 4);
        gp_ = (float*)c.take((int64_t)B * P * 4);
        xemb_ = (float*)c.take((int64_t)B * P * 4);
        fecur_ = (float*)c.take((int64_t)B * P * 4);
        jpart_ = (float4*)c.take((int64_t)B * joint_tiles_ * 16);
        dur_ = (float*)c.take((int64_t)B * dm_.n_dur * 4);
        out_tok_ = (int*)c.take((int64_t)B * cap_ * 4);
        out_frame_ = (int*)c.take((int64_t)B * cap_ * 4);
        out_t1_ = (float*)c.take((int64_t)B * cap_ * 4);
        out_t2_ = (float*)c.take((int64_t)B * cap_ * 4);
        dsum_ = (double*)c.take(16);
        if (!pass) {
            abytes_ = c.off;
            if (hipMalloc(&aarena_, abytes_) != hipSuccess) {
                aarena_ = nullptr;
                throw std::runtime_error("out of device memory for workspace (" + std::to_string(abytes_) + " B)");
            }
            HIP_CHECK(hipMemsetAsync(aarena_, 0, abytes_, st_));
        }
    }
}

void ParakeetEngine::upload_tables() {
    std::vector<float> win(PK_NFFT), basis((size_t)PK_DFT_N * PK_NFFT, 0.0f), fb, fbT;
    for (int i = 0; i < PK_NFFT; i++) {
        const int j = i - (PK_NFFT - 400) / 2;  // the 400-sample symmetric Hann window centred in 512
        win[i] = (j >= 0 && j < 400) ? (float)(0.5 - 0.5 * cos(2.0 * M_PI * j / 399.0)) : 0.0f;
    }
    for (int k = 0; k < PK_NBIN; ++k)
        for (int i = 0; i < PK_NFFT; ++i) {
            const int ph = (k * i) & (PK_NFFT - 1);
            basis[(size_t)k * PK_NFFT + i] = (float)cos(2.0 * M_PI * ph / PK_NFFT);
            basis[(size_t)(PK_NBIN + k) * PK_NFFT + i] = (float)sin(2.0 * M_PI * ph / PK_NFFT);
        }
    slaney_filters(dm_.n_mels, &fb);
    fbT.resize(fb.size());
    for (int j = 0; j < dm_.n_mels; ++j)
        for (int k = 0; k < PK_NBIN; ++k) fbT[(size_t)k * dm_.n_mels + j] = fb[(size_t)j * PK_NBIN + k];
    HIP_CHECK(hipMalloc(&win_, win.size() * 4));
    HIP_CHECK(hipMalloc(&basis_, basis.size() * 4));
    HIP_CHECK(hipMalloc(&fbT_, fbT.size() * 4));
    HIP_CHECK(hipMemcpy(win_, win.data(), win.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(basis_, basis.data(), basis.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(fbT_, fbT.data(), fbT.size() * 4, hipMemcpyHostToDevice));
}

void ParakeetEngine::frame_counts(const int* n, int B, std::vector<int>* lens, int* Tp, int* T1p, int* T2p,
                                  int* T3p) const {
    lens->assign((size_t)B * 4, 0);
    int tp = 1;
    for (int b = 0; b < B; ++b) {
        if (n[b] < 0 || n[b] > max_samples_) throw std::runtime_error("utterance length out of range");
        // valid frames: NeMo FilterbankFeatures.get_seq_len = n / hop (HF feature_extraction_parakeet.py:263);
        // the STFT's last centred frame is not one of them.  Under 160 samples nothing is decoded.
        const int T = n[b] / PK_HOP;
        (*lens)[b * 4 + 0] = T;
        (*lens)[b * 4 + 1] = sub_len(T);
        (*lens)[b * 4 + 2] = sub_len(sub_len(T));
        (*lens)[b * 4 + 3] = sub_len(sub_len(sub_len(T)));
        tp = std::max(tp, T);
    }
    *Tp = tp;
    *T1p = halve(tp);
    *T2p = halve(*T1p);
    *T3p = halve(*T2p);
}

void ParakeetEngine::run_mel(const float* pcm_dev, int64_t stride, int B, int Tp) {
    pk_frames(pcm_dev, stride, nsamp_, B, Tp, win_, frames_, st_);
    GemmArgs g{};
    g.A = frames_; g.lda = PK_NFFT;
    g.W = basis_; g.ldw = PK_NFFT;
    g.M = B * Tp; g.N = PK_DFT_N; g.K = PK_NFFT;
    g.C = spec_; g.ldc = PK_DFT_N;
    gemm_nt(DT_F32, EPI_BIAS, g, 1, st_);
    SPT_LAUNCH_CHECK();
    pk_melpow(spec_, B * Tp, fbT_, dm_.n_mels, mel_, st_);
    pk_mel_norm(mel_, lens_, B, Tp, dm_.n_mels, st_);
}

// GEMM tile choice: the 256 x 256 tile whenever at least ~128 of its workgroups are in flight
// (its MFMA efficiency beats the smaller tiles' even with part of the chip idle), else the 64 x 128
// tile from two workgroups per CU up, else the 64 x 64 one (several waves per SIMD cover each
// other's LDS reads and slab waits; r3 exp_r3v / exp_r3y / exp_r3z: 20-45 % faster than the
// 128 x 128 tile at M = 832 and M = 3000, bitwise equal; the 128 x 128 tile stays for f32).
// Residual products (EPI_PARTIAL, N = d) also split K over grid.y toward ~192 (256-tile), ~512
// (128 / 64 x 128) or ~1024 (64 x 64) workgroups, keeping >= 8 K-steps per split;
// their f32 slabs are summed, with the bias and the 1/2 FFN scale, by the next LayerNorm.
// Returns the split used.
int ParakeetEngine::gemm(int dt, int epi, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                         const float* bias, void* Cp, int ldc, float alpha) {
    // SPT_GEMM_T256 / SPT_GEMM_T64 / SPT_NO_SKINNY: read per call so tests can pin each variant
    // (eager calls only: a captured encoder graph keeps the variants it was captured with)
    const char* t256e = getenv("SPT_GEMM_T256");
    const int t256 = t256e ? atoi(t256e) : 128;
    const char* t64e = getenv("SPT_GEMM_T64");
    const bool t64_ok = !(t64e && atoi(t64e) == 0);
    const bool no_skinny = getenv("SPT_NO_SKINNY") != nullptr;
    int variant = 1, ks = 1;
    if (dt != DT_F32 && M <= 64 && N % 16 == 0 && K % 128 == 0 && !no_skinny) {
        // skinny: >= 256 workgroups of 16 columns (residual products split K to get there)
        variant = 3;
        if (epi == EPI_PARTIAL)
            while (ks < 8 && (N / 16) * ks < 256 && K % (2 * ks) == 0 && (K / (2 * ks)) % 128 == 0) ks *= 2;
    } else if (dt != DT_F32 && N % 256 == 0 && K % 64 == 0 && !(t64_ok && (int64_t)cdiv(M, 256) * (N / 256) < 32)) {
        const int64_t t = (int64_t)cdiv(M, 256) * (N / 256);
        int k2 = 1;
        if (epi == EPI_PARTIAL)
            while (k2 < 8 && t * k2 < 192 && K % (2 * k2) == 0 && (K / (2 * k2)) % 64 == 0 && K / (2 * k2) >= 512) k2 *= 2;
        if (t * k2 >= t256) { variant = 2; ks = k2; }
    }
    if (variant == 1 && dt != DT_F32 && M > 64 && t64_ok) variant = (int64_t)cdiv(M, 64) * (N / 128) >= 512 ? 4 : 5;
    if (variant == 1 && epi == EPI_PARTIAL) {
        const int64_t t = (int64_t)cdiv(M, 128) * (N / 128);
        while (ks < 8 && t * ks * 2 <= 512 && K % (2 * ks) == 0 && (K / (2 * ks)) % 64 == 0) ks *= 2;
    } else if ((variant == 4 || variant == 5) && epi == EPI_PARTIAL) {
        const int64_t t = (int64_t)cdiv(M, 64) * (N / (variant == 4 ? 128 : 64));
        const int64_t cap = variant == 4 ? 512 : 1024;
        while (ks < 8 && t * ks * 2 <= cap && K % (2 * ks) == 0 && K / (2 * ks) >= 512 && (K / (2 * ks)) % 64 == 0) ks *= 2;
    }
    GemmArgs g{};
    g.A = A; g.lda = lda; g.W = W; g.ldw = ldw; g.M = M; g.N = N; g.K = K; g.bias = bias;
    g.C = Cp; g.ldc = ldc; g.alpha = alpha; g.ksplit = ks; g.c_split = (int64_t)M * ldc;
    gemm_nt_variant(dt, epi, g, 1, variant, st_);
    SPT_LAUNCH_CHECK();
    return ks;
}

void ParakeetEngine::run_encoder(int B, int Tp, int T1p, int T2p, int T3p) {
    const int C = dm_.sub_ch, d = dm_.d, H = dm_.n_heads, dk = d / H, ff = dm_.ff, Ln = dm_.n_layers;
    // ---- dw_striding subsampling (channel-last activations)
    pk_conv0(dt_, mel_, lens_, B, Tp, dm_.n_mels, c0_w_, c0_b_, C, y1_, T1p, F1_, st_);
    pk_dwconv(dt_, y1_, lens_, 1, B, T1p, F1_, dw1_w_, dw1_b_, C, y2a_, T2p, F2_, st_);
    gemm(dt_, EPI_BIAS_RELU, y2a_, C, pw1_w_, C, B * T2p * F2_, C, C, pw1_b_, y2_, C);
    pk_dwconv(dt_, y2_, lens_, 2, B, T2p, F2_, dw2_w_, dw2_b_, C, y3a_, T3p, F3_, st_);
    gemm(dt_, EPI_BIAS_RELU, y3a_, C, pw2_w_, C, B * T3p * F3_, C, C, pw2_b_, y3_, C);
    float* x = x_;
    float* x2 = x_ + (int64_t)max_batch_ * T3max_ * d;
    const int M = B * T3p;
    gemm(dt_, EPI_BIAS_F32, y3_, F3_ * C, sub_w_, F3_ * C, M, d, F3_ * C, sub_b_, x, d, sqrtf((float)d));
    mark(PK_ST_SUB);
    // ---- relative positions, projected for every layer at once
    pk_relpos(dt_, T3p, d, pe_, st_);
    gemm(dt_, EPI_BIAS, pe_, d, pos_w_, d, 2 * T3p - 1, Ln * d, d, nullptr, pp_, Ln * d);
    mark(PK_ST_POS);
    const int64_t sst = (int64_t)M * d;
    int ks;
    for (int l = 0; l < Ln; ++l) {
        const Layer& y = L_[l];
        // 1/2 FFN; its product stays pending in the slabs until the next LayerNorm (the first
        // block's input LayerNorm here, the others' in the previous block's output LayerNorm)
        if (l == 0) {
            layernorm(dt_, x, M, d, y.ln1_w, y.ln1_b, xn_, st_);
            mark(PK_ST_LN);
        }
        gemm(dt_, EPI_BIAS_SWISH, xn_, d, y.ff1_w1, d, M, ff, d, y.ff1_b1, ffh_, ff);
        ks = gemm(dt_, EPI_PARTIAL, ffh_, ff, y.ff1_w2, ff, M, d, ff, nullptr, slab_, d);
        mark(PK_ST_FFN);
        // rel-pos MHSA
        layernorm_pend(dt_, x, M, d, slab_, ks, sst, y.ff1_b2, 0.5f, y.lna_w, y.lna_b, xn_, true, st_);
        mark(PK_ST_LN);
        gemm(dt_, EPI_BIAS, xn_, d, y.qkv_w, d, M, 3 * d, d, y.qkv_b, qkv_, 3 * d);
        mark(PK_ST_QKVO);
        pk_rel_attn(dt_, qkv_, (const char*)pp_ + (size_t)l * d * esz_, Ln * d, y.pos_u, y.pos_v, lens_, B, T3p, H, dk,
                    ctx_, st_);
        mark(PK_ST_ATTN);
        ks = gemm(dt_, EPI_PARTIAL, ctx_, d, y.o_w, d, M, d, d, nullptr, slab_, d);
        mark(PK_ST_QKVO);
        // convolution module
        layernorm_pend(dt_, x, M, d, slab_, ks, sst, y.o_b, 1.0f, y.lnc_w, y.lnc_b, xn_, true, st_);
        mark(PK_ST_LN);
        gemm(dt_, EPI_BIAS, xn_, d, y.pw1_w, d, M, 2 * d, d, y.pw1_b, glu_, 2 * d);
        mark(PK_ST_CONV_PW);
        pk_conv_module(dt_, glu_, lens_, B, T3p, d, dm_.conv_k, y.dw_w, y.dw_b, y.bn_g, y.bn_b, y.bn_m, y.bn_v, cv_, st_);
        mark(PK_ST_CONV_DW);
        ks = gemm(dt_, EPI_PARTIAL, cv_, d, y.pw2_w, d, M, d, d, nullptr, slab_, d);
        mark(PK_ST_CONV_PW);
        // 1/2 FFN
        layernorm_pend(dt_, x, M, d, slab_, ks, sst, y.pw2_b, 1.0f, y.ln2_w, y.ln2_b, xn_, true, st_);
        mark(PK_ST_LN);
        gemm(dt_, EPI_BIAS_SWISH, xn_, d, y.ff2_w1, d, M, ff, d, y.ff2_b1, ffh_, ff);
        ks = gemm(dt_, EPI_PARTIAL, ffh_, ff, y.ff2_w2, ff, M, d, ff, nullptr, slab_, d);
        mark(PK_ST_FFN);
        // LayerNorm out (f32) of x + the pending 1/2 FFN into the other residual buffer, and with
        // it the next block's input LayerNorm
        if (l + 1 < Ln)
            layernorm_pend2(dt_, x, M, d, slab_, ks, sst, y.ff2_b2, 0.5f, y.lno_w, y.lno_b, x2, L_[l + 1].ln1_w,
                            L_[l + 1].ln1_b, xn_, st_);
        else
            layernorm_pend(DT_F32, x, M, d, slab_, ks, sst, y.ff2_b2, 0.5f, y.lno_w, y.lno_b, x2, false, st_);
        mark(PK_ST_LN);
        std::swap(x, x2);
    }
    // the joint's encoder projection of every frame (f32)
    gemm(DT_F32, EPI_BIAS, x, d, jenc_w_, d, M, dm_.pred, d, jenc_b_, fe_, dm_.pred);
    mark(PK_ST_JOINT);
    enc_out_ = x;
}

// The encoder's ~16 launches per layer replayed as one hipGraph per (batch, padded frames) once
// that shape has been seen twice (a stream of fixed windows, a batch of full chunks); shapes seen
// once run eagerly, so arbitrary utterance lengths do not pay for graph instantiation.
void ParakeetEngine::encode(int B, int Tp, int T1p, int T2p, int T3p) {
    static const bool no_graph = getenv("SPT_NO_GRAPH") != nullptr;
    const std::pair<int, int> key{B, Tp};
    auto it = enc_graphs_.find(key);
    if (it == enc_graphs_.end() && !no_graph && enc_seen_[key]++ >= 1 && enc_graphs_.size() < 32) {
        hipGraph_t graph;
        HIP_CHECK(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal));
        run_encoder(B, Tp, T1p, T2p, T3p);
        HIP_CHECK(hipStreamEndCapture(st_, &graph));
        hipGraphExec_t exec;
        HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        HIP_CHECK(hipGraphDestroy(graph));
        it = enc_graphs_.emplace(key, exec).first;
        enc_out_graph_[key] = enc_out_;
    }
    if (it != enc_graphs_.end()) {
        HIP_CHECK(hipGraphLaunch(it->second, st_));
        enc_out_ = enc_out_graph_[key];
    } else {
        run_encoder(B, Tp, T1p, T2p, T3p);
    }
}

void ParakeetEngine::mark(int cls) {
    if (!prof_on_) return;
    const size_t i = prof_cls_.size();
    if (i >= prof_ev_.size()) throw std::runtime_error("profile_encoder: event pool exhausted");
    HIP_CHECK(hipEventRecord(prof_ev_[i], st_));
    prof_cls_.push_back(cls);
}

void ParakeetEngine::profile_encoder(int iters, double ms[PK_ST_COUNT]) {
    select();
    const int B = last_dims_[0];
    if (B < 1 || !enc_out_) throw std::runtime_error("profile_encoder needs a completed transcription call first");
    if (iters < 1 || iters > 1000) throw std::runtime_error("iters out of range");
    const size_t need = (size_t)14 * dm_.n_layers + 8;  // 13 marks per layer
    while (prof_ev_.size() < need) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        prof_ev_.push_back(e);
    }
    for (int c = 0; c < PK_ST_COUNT; ++c) ms[c] = 0.0;
    for (int it = 0; it < iters; ++it) {
        prof_cls_.clear();
        prof_on_ = true;
        HIP_CHECK(hipEventRecord(ev_[0], st_));
        try {
            run_encoder(B, last_dims_[1], last_dims_[2], last_dims_[3], last_dims_[4]);
        } catch (...) {
            prof_on_ = false;
            throw;
        }
        prof_on_ = false;
        HIP_CHECK(hipStreamSynchronize(st_));
        hipEvent_t prev = ev_[0];
        for (size_t i = 0; i < prof_cls_.size(); ++i) {
            float t = 0.f;
            HIP_CHECK(hipEventElapsedTime(&t, prev, prof_ev_[i]));
            ms[prof_cls_[i]] += t;
            prev = prof_ev_[i];
        }
    }
    for (int c = 0; c < PK_ST_COUNT; ++c) ms[c] /= iters;
}

void ParakeetEngine::enqueue_step(int B, int max_symbols, int cap, int parity) {
    const int P = dm_.pred;
    const size_t BP = (size_t)B * P;
    auto hbuf = [&](float* base, int layer, int par) { return base + ((size_t)layer * 2 + par) * BP; };
    const int p = parity, q = parity ^ 1;
    PkDecArgs a{};
    a.B = B; a.P = P; a.V = dm_.n_vocab; a.n_dur = dm_.n_dur; a.st = state_;
    // LSTM layer 0: x = [emb(token) | h0]
    a.WT = lstm_wt_[0]; a.ld = 4 * P; a.K = 2 * P; a.N = 4 * P; a.b0 = lstm_bih_[0]; a.b1 = lstm_bhh_[0];
    a.xin = xemb_; a.h_in = hbuf(h_, 0, p); a.c_in = hbuf(c_, 0, p); a.h_out = hbuf(h_, 0, q); a.c_out = hbuf(c_, 0, q);
    pk_decode_stage(PKD_LSTM, a, st_);
    // LSTM layer 1: x = [h0' | h1]
    a.WT = lstm_wt_[1]; a.b0 = lstm_bih_[1]; a.b1 = lstm_bhh_[1]; a.xin = hbuf(h_, 0, q);
    a.h_in = hbuf(h_, 1, p); a.c_in = hbuf(c_, 1, p); a.h_out = hbuf(h_, 1, q); a.c_out = hbuf(c_, 1, q);
    pk_decode_stage(PKD_LSTM, a, st_);
    // prediction projection of h1' (rows with a new token)
    a.WT = jpred_wt_; a.ld = P_pad_; a.K = P; a.N = P; a.b0 = jpred_b_; a.b1 = nullptr; a.xin = hbuf(h_, 1, q); a.gp = gp_;
    pk_decode_stage(PKD_PRED, a, st_);
    // joint: ReLU(enc[t] + pred) -> logits -> per-workgroup top-2 + durations
    a.WT = jout_wt_; a.ld = joint_pad_; a.K = P; a.N = dm_.n_vocab + 1 + dm_.n_dur; a.b0 = jout_b_;
    a.fe = fecur_; a.part = jpart_; a.n_tiles = joint_tiles_; a.dur = dur_;
    pk_decode_stage(PKD_JOINT, a, st_);
    PkFinArgs f{};
    f.part = jpart_; f.n_tiles = joint_tiles_; f.dur = dur_;
    f.V = dm_.n_vocab; f.n_dur = dm_.n_dur; f.max_symbols = max_symbols; f.B = B; f.cap = cap; f.lens = lens_;
    f.st = state_; f.out_tok = out_tok_; f.out_frame = out_frame_; f.out_t1 = out_t1_; f.out_t2 = out_t2_;
    f.P = P; f.emb = emb_; f.fe = fe_; f.xemb = xemb_; f.fecur = fecur_;
    pk_joint_fin(f, st_);
}

void ParakeetEngine::run_decode(int B, int T3p, int max_symbols, std::vector<PkUtt>* out) {
    const int P = dm_.pred;
    pk_state_init(state_, B, dm_.n_vocab, h_, c_, 4 * B * P, xemb_, fecur_, fe_, lens_, T3p, P, st_);
    const GraphKey key{B, max_symbols};  // the frame stride lives in the state rows
    auto it = graphs_.find(key);
    static const bool no_graph = getenv("SPT_NO_GRAPH") != nullptr;
    if (it == graphs_.end() && !no_graph) {
        hipGraph_t graph;
        HIP_CHECK(hipStreamBeginCapture(st_, hipStreamCaptureModeThreadLocal));
        for (int s = 0; s < kStepsPerGraph; ++s) enqueue_step(B, max_symbols, cap_, s & 1);
        HIP_CHECK(hipStreamEndCapture(st_, &graph));
        hipGraphExec_t exec;
        HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        HIP_CHECK(hipGraphDestroy(graph));
        it = graphs_.emplace(key, exec).first;
    }
    // every joint evaluation advances a frame or emits one of <= max_symbols tokens of it
    const int max_steps = T3p * (max_symbols + 1) + kStepsPerGraph;
    // read-backs into pinned memory: the state after every graph, then only the emitted prefix of
    // each output row (r6: four whole [B][cap] pageable copies -- 6 MB at B = 64 -- cost the C5
    // call more host time than its decoder's GPU time)
    if (B > hst_cap_) {
        if (hst_pin_) HIP_CHECK(hipHostFree(hst_pin_));
        hst_pin_ = nullptr;
        hst_cap_ = 0;
        HIP_CHECK(hipHostMalloc((void**)&hst_pin_, (size_t)B * sizeof(PkState), hipHostMallocDefault));
        hst_cap_ = B;
    }
    int steps = 0;
    while (true) {
        if (no_graph) for (int s = 0; s < kStepsPerGraph; ++s) enqueue_step(B, max_symbols, cap_, s & 1);
        else HIP_CHECK(hipGraphLaunch(it->second, st_));
        steps += kStepsPerGraph;
        HIP_CHECK(hipMemcpyAsync(hst_pin_, state_, B * sizeof(PkState), hipMemcpyDeviceToHost, st_));
        HIP_CHECK(hipStreamSynchronize(st_));
        bool all = true;
        for (int b = 0; b < B; ++b) all = all && hst_pin_[b].done;
        if (all) break;
        if (steps > max_steps) throw std::runtime_error("TDT decoding did not finish (internal error)");
    }
    hstate_.assign(hst_pin_, hst_pin_ + B);
    tm_.n_steps = steps;
    HIP_CHECK(hipEventRecord(ev_[3], st_));
    int nmo = 0;  // the longest emitted row
    for (int b = 0; b < B; ++b) nmo = std::max(nmo, std::min(hstate_[b].n_out, cap_));
    out->assign(B, PkUtt{});
    if (nmo == 0) return;
    const size_t per = (size_t)B * nmo;  // one output's trimmed rows
    if (4 * per > res_cap_) {
        if (res_pin_) HIP_CHECK(hipHostFree(res_pin_));
        res_pin_ = nullptr;
        res_cap_ = 0;
        HIP_CHECK(hipHostMalloc((void**)&res_pin_, 4 * per * 4, hipHostMallocDefault));
        res_cap_ = 4 * per;
    }
    const void* src[4] = {out_tok_, out_frame_, out_t1_, out_t2_};
    for (int k = 0; k < 4; ++k)
        HIP_CHECK(hipMemcpy2DAsync(res_pin_ + k * per, (size_t)nmo * 4, src[k], (size_t)cap_ * 4, (size_t)nmo * 4, B,
                                   hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    const int* tok = res_pin_;
    const int* fr = res_pin_ + per;
    const float* t1 = (const float*)(res_pin_ + 2 * per);
    const float* t2 = (const float*)(res_pin_ + 3 * per);
    for (int b = 0; b < B; ++b) {
        const int n = std::min(hstate_[b].n_out, cap_);
        PkUtt& u = (*out)[b];
        const size_t o = (size_t)b * nmo;
        u.tok.assign(tok + o, tok + o + n);
        u.frame.assign(fr + o, fr + o + n);
        u.top1.assign(t1 + o, t1 + o + n);
        u.top2.assign(t2 + o, t2 + o + n);
    }
}

void ParakeetEngine::transcribe_device(const float* pcm_dev, int64_t stride, const int* n, int B, int max_symbols,
                                       std::vector<PkUtt>* out) {
    if (B < 1 || B > max_batch_) throw std::runtime_error("batch must be in [1, max_batch]");
    if (max_symbols < 1 || max_symbols > kMaxSymbols) throw std::runtime_error("max_symbols must be in [1, 16]");
    if (B > 1)
        for (int b = 0; b < B; ++b)
            if (stride < n[b]) throw std::runtime_error("device stride shorter than an utterance");
    select();
    std::vector<int> lens;
    int Tp, T1p, T2p, T3p;
    frame_counts(n, B, &lens, &Tp, &T1p, &T2p, &T3p);
    last_lens_ = lens;
    last_T3p_ = T3p;
    last_dims_[0] = B; last_dims_[1] = Tp; last_dims_[2] = T1p; last_dims_[3] = T2p; last_dims_[4] = T3p;
    HIP_CHECK(hipEventRecord(ev_[0], st_));
    HIP_CHECK(hipMemcpyAsync(nsamp_, n, B * 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(lens_, lens.data(), lens.size() * 4, hipMemcpyHostToDevice, st_));
    run_mel(pcm_dev, stride, B, Tp);
    HIP_CHECK(hipEventRecord(ev_[1], st_));
    encode(B, Tp, T1p, T2p, T3p);
    HIP_CHECK(hipEventRecord(ev_[2], st_));
    run_decode(B, T3p, max_symbols, out);
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1])); tm_.mel_ms = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[1], ev_[2])); tm_.encoder_ms = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[2], ev_[3])); tm_.decode_ms = ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[3])); tm_.total_ms = ms;
    tm_.batch = B;
    tm_.enc_frames = T3p;
}

void ParakeetEngine::transcribe_host(const float* const* pcm, const int* n, int B, int max_symbols,
                                     std::vector<PkUtt>* out) {
    if (B < 1 || B > max_batch_) throw std::runtime_error("batch must be in [1, max_batch]");
    select();
    int nmax = 0;
    for (int b = 0; b < B; ++b) {
        if (n[b] < 0 || n[b] > max_samples_) throw std::runtime_error("utterance length out of range");
        if (n[b] > 0 && !pcm[b]) throw std::runtime_error("null pcm");
        nmax = std::max(nmax, n[b]);
    }
    // Many short windows (C5: 64 x 1 s) paid a pageable copy each (0.68 ms for 4 MB): windows of
    // up to 4 s are gathered into pinned rows of nmax samples and sent by one 2D copy (the tail of
    // a shorter row is never read: the front end stops at n[b]).  Longer windows keep the pageable
    // copies (8 x 30 s: the host gather cost more than it saved).  SPT_PK_PINNED=0: never, 2: always.
    // h2d_ms = the host gather + the copy on the stream.
    const int pin_env = getenv("SPT_PK_PINNED") ? atoi(getenv("SPT_PK_PINNED")) : 1;
    const bool pinned = pin_env == 2 || (pin_env != 0 && nmax <= 4 * 16000);
    double gather_ms = 0.0;
    if (pinned && nmax > 0) {
        const size_t need = (size_t)B * nmax;
        if (need > pin_cap_) {
            if (pin_) HIP_CHECK(hipHostFree(pin_));
            pin_ = nullptr;
            pin_cap_ = 0;
            HIP_CHECK(hipHostMalloc((void**)&pin_, need * 4, hipHostMallocDefault));
            pin_cap_ = need;
        }
        // the previous call's copy out of pin_ has completed (calls end by reading their results
        // back on st_; this also covers one that threw part way)
        HIP_CHECK(hipStreamSynchronize(st_));
        const auto t0 = std::chrono::steady_clock::now();
        for (int b = 0; b < B; ++b)
            if (n[b]) memcpy(pin_ + (size_t)b * nmax, pcm[b], (size_t)n[b] * 4);
        gather_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        HIP_CHECK(hipEventRecord(ev_[4], st_));
        HIP_CHECK(hipMemcpy2DAsync(pcm_, (size_t)max_samples_ * 4, pin_, (size_t)nmax * 4, (size_t)nmax * 4, B,
                                   hipMemcpyHostToDevice, st_));
    } else {
        HIP_CHECK(hipEventRecord(ev_[4], st_));
        for (int b = 0; b < B; ++b)
            if (n[b]) HIP_CHECK(hipMemcpyAsync(pcm_ + (size_t)b * max_samples_, pcm[b], (size_t)n[b] * 4, hipMemcpyHostToDevice, st_));
    }
    HIP_CHECK(hipEventRecord(ev_[5], st_));
    transcribe_device(pcm_, max_samples_, n, B, max_symbols, out);
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[4], ev_[5]));
    tm_.h2d_ms = ms + gather_ms;
}

void ParakeetEngine::debug_mel(const float* pcm_host, int n, float* out_host) {
    select();
    if (n < 0 || n > max_samples_) throw std::runtime_error("utterance length out of range");
    std::vector<int> lens;
    int Tp, T1p, T2p, T3p;
    frame_counts(&n, 1, &lens, &Tp, &T1p, &T2p, &T3p);
    if (n) HIP_CHECK(hipMemcpyAsync(pcm_, pcm_host, (size_t)n * 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(nsamp_, &n, 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(lens_, lens.data(), 16, hipMemcpyHostToDevice, st_));
    run_mel(pcm_, max_samples_, 1, Tp);
    std::vector<float> tmp((size_t)Tp * dm_.n_mels);
    HIP_CHECK(hipMemcpyAsync(tmp.data(), mel_, tmp.size() * 4, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    for (int t = 0; t < Tp; ++t)
        for (int j = 0; j < dm_.n_mels; ++j) out_host[(size_t)j * Tp + t] = tmp[(size_t)t * dm_.n_mels + j];
}

void ParakeetEngine::debug_encode(const float* mel_host, int T, float* out_host) {
    select();
    if (T < 1 || T > Tmax_) throw std::runtime_error("mel frame count out of range");
    const int T1 = halve(T), T2 = halve(T1), T3 = halve(T2);
    const int lens[4] = {T, T1, T2, T3};
    std::vector<float> tmp((size_t)T * dm_.n_mels);
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < dm_.n_mels; ++j) tmp[(size_t)t * dm_.n_mels + j] = mel_host[(size_t)j * T + t];
    HIP_CHECK(hipMemcpyAsync(lens_, lens, 16, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(mel_, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, st_));
    run_encoder(1, T, T1, T2, T3);
    HIP_CHECK(hipMemcpyAsync(out_host, enc_out_, (size_t)T3 * dm_.d * 4, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
}

int ParakeetEngine::debug_last_encoder(int b, float* out_host) {
    select();
    if (!enc_out_ || last_lens_.empty()) throw std::runtime_error("no completed transcription call");
    if (b < 0 || (size_t)b * 4 >= last_lens_.size()) throw std::runtime_error("no such row in the last call");
    const int T3 = last_lens_[b * 4 + 3];
    HIP_CHECK(hipStreamSynchronize(st_));
    if (T3 > 0)
        HIP_CHECK(hipMemcpy(out_host, enc_out_ + (size_t)b * last_T3p_ * dm_.d, (size_t)T3 * dm_.d * 4,
                            hipMemcpyDeviceToHost));
    return T3;
}

void ParakeetEngine::debug_decode(const float* enc_host, int T3, int max_symbols, PkUtt* out) {
    select();
    if (T3 < 1 || T3 > T3max_) throw std::runtime_error("encoder frame count out of range");
    if (max_symbols < 1 || max_symbols > kMaxSymbols) throw std::runtime_error("max_symbols must be in [1, 16]");
    const int lens[4] = {0, 0, 0, T3};
    HIP_CHECK(hipMemcpyAsync(lens_, lens, 16, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipMemcpyAsync(x_, enc_host, (size_t)T3 * dm_.d * 4, hipMemcpyHostToDevice, st_));
    GemmArgs g{};
    g.A = x_; g.lda = dm_.d; g.W = jenc_w_; g.ldw = dm_.d; g.M = T3; g.N = dm_.pred; g.K = dm_.d;
    g.bias = jenc_b_; g.C = fe_; g.ldc = dm_.pred;
    gemm_nt(DT_F32, EPI_BIAS, g, 1, st_);
    SPT_LAUNCH_CHECK();
    HIP_CHECK(hipEventRecord(ev_[2], st_));
    std::vector<PkUtt> res;
    run_decode(1, T3, max_symbols, &res);
    *out = res[0];
}

bool ParakeetEngine::debug_weight_checksum(int tid, double* out2) {
    auto it = table_.find(tid);
    if (it == table_.end()) return false;
    const TSpec& t = specs_[it->second];
    if (t.mode == PK_PLACE_TRANSPOSE || t.mode == PK_PLACE_LSTM || t.mode == PK_PLACE_BLOCKED) return false;  // re-tiled
    select();
    HIP_CHECK(hipMemsetAsync(dsum_, 0, 16, st_));
    tensor_checksum(t.dt, t.dst, t.n, dsum_, st_);
    HIP_CHECK(hipMemcpyAsync(out2, dsum_, 16, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    return true;
}

}  // namespace spt
