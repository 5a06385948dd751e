// vad.hip -- Silero VAD v4 + SmoothedVad on the device (see vad.h).
//
// The weights are read from the app's own model file (resources/models/silero_vad_v4.onnx) by the
// ONNX reader (onnx_pb.cpp): the 16 kHz branch of the graph's top-level If (sr == 16000), its
// Conv nodes in graph order, and the two LSTM nodes of the branch that takes the caller's state.
#include "vad.h"

#include <cmath>
#include <cstring>
#include <stdexcept>

#include "common.h"
#include "onnx_pb.h"

namespace spt {

constexpr int kPadL = 96;      // reflect padding of the frame on both sides (the graph's Pad)
constexpr int kPadded = kVadFrame + 2 * kPadL;  // 672
constexpr int kT = 7;          // STFT steps: (672 - 256) / 64 + 1

// ------------------------------------------------------------------ model (host)
struct ConvW {  // one Conv node: weight [out][in / group][k], bias [out]
    int out = 0, in_g = 0, k = 0, group = 1, stride = 1, pad = 0;
    std::vector<float> w, b;
};
struct SileroHost {
    ConvW stft, filt;                 // forward basis (258 x 256, stride 64), adaptive-normalisation filter (7)
    ConvW blk[17];                    // the encoder's convolutions in graph order (below)
    ConvW dec;                        // decoder 1x1 conv 64 -> 1
    std::vector<float> lw[2], lr[2], lb[2];  // LSTM layers: W [256][64], R [256][64], B [512] (ONNX gates i, o, f, c)
    float pad_left = 96.f, pad_right = 96.f, mag_scale = 1048576.f;
};

namespace {

const onnx::Tensor* find_t(const std::vector<const onnx::Graph*>& scopes, const std::string& name) {
    for (auto it = scopes.rbegin(); it != scopes.rend(); ++it)
        if (const onnx::Tensor* t = (*it)->find(name)) return t;
    return nullptr;
}

std::vector<float> vals(const std::vector<const onnx::Graph*>& scopes, const std::string& name, std::string* err) {
    const onnx::Tensor* t = find_t(scopes, name);
    std::vector<float> v;
    if (!t) { *err = "Silero model: no initializer '" + name + "'"; return v; }
    if (!t->to_f32(&v, err)) v.clear();
    return v;
}

bool read_conv(const onnx::Node& n, const std::vector<const onnx::Graph*>& sc, ConvW* c, std::string* err) {
    const onnx::Tensor* w = n.inputs.size() > 1 ? find_t(sc, n.inputs[1]) : nullptr;
    if (!w || w->dims.size() != 3) { *err = "Silero model: Conv '" + n.name + "' weight is not a 1-D conv initializer"; return false; }
    c->out = (int)w->dims[0]; c->in_g = (int)w->dims[1]; c->k = (int)w->dims[2];
    if (const onnx::Attribute* a = n.attr("group")) c->group = (int)a->i;
    if (const onnx::Attribute* a = n.attr("strides"); a && !a->ints.empty()) c->stride = (int)a->ints[0];
    if (const onnx::Attribute* a = n.attr("pads"); a && !a->ints.empty()) c->pad = (int)a->ints[0];
    if (!w->to_f32(&c->w, err)) return false;
    if (n.inputs.size() > 2 && !n.inputs[2].empty()) {
        c->b = vals(sc, n.inputs[2], err);
        if (c->b.empty()) return false;
    } else c->b.assign(c->out, 0.f);
    return (int)c->b.size() == c->out;
}

const onnx::Graph* branch(const onnx::Node& n, const char* which) {
    const onnx::Attribute* a = n.attr(which);
    return a ? a->g.get() : nullptr;
}

// expected encoder conv shapes (out, in/group, k, group, stride) in graph order
struct Shape { int out, in_g, k, group, stride; };
const Shape kBlk[17] = {
    {258, 1, 5, 258, 1}, {16, 258, 1, 1, 1}, {16, 258, 1, 1, 1},   // first_layer: dw, pw, proj
    {16, 16, 1, 1, 2},                                              // stride-2 1x1
    {16, 1, 5, 16, 1}, {32, 16, 1, 1, 1}, {32, 16, 1, 1, 1},       // encoder.3: dw, pw, proj
    {32, 32, 1, 1, 2},
    {32, 1, 5, 32, 1}, {32, 32, 1, 1, 1},                           // encoder.7: dw, pw (identity residual)
    {32, 32, 1, 1, 2},
    {32, 1, 5, 32, 1}, {64, 32, 1, 1, 1}, {64, 32, 1, 1, 1},       // encoder.11: dw, pw, proj
    {64, 64, 1, 1, 1},                                              // 1x1 before the LSTM
    {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}};
constexpr int kNBlk = 15;

bool load_silero(const std::string& path, SileroHost* m, std::string* err) {
    onnx::Model model;
    if (!model.open(path, err)) return false;
    const onnx::Graph& top = model.graph();
    // the top-level If on sr == 16000: its then branch is the 16 kHz model
    const onnx::Graph* g16 = nullptr;
    for (const onnx::Node& n : top.nodes)
        if (n.op_type == "If") g16 = branch(n, "then_branch");
    if (!g16) { *err = path + ": not the Silero VAD graph (no sample-rate If)"; return false; }
    std::vector<const onnx::Graph*> sc{&top, g16};
    std::vector<const onnx::Node*> convs;
    const onnx::Node* lstm_if = nullptr;
    for (const onnx::Node& n : g16->nodes) {
        if (n.op_type == "Conv") convs.push_back(&n);
        if (n.op_type == "If")
            if (const onnx::Graph* t = branch(n, "then_branch"))
                for (const onnx::Node& x : t->nodes)
                    if (x.op_type == "LSTM") lstm_if = &n;
        if (n.op_type == "Pad" && n.inputs.size() > 1) {
            std::vector<float> p = vals(sc, n.inputs[1], err);
            if (p.size() >= 2 && p.size() % 2 == 0) {  // [begins..., ends...]: the time (last) axis
                m->pad_left = p[p.size() / 2 - 1];
                m->pad_right = p[p.size() - 1];
            }
        }
        if (n.op_type == "Mul")
            for (const std::string& in : n.inputs)
                if (const onnx::Tensor* t = find_t(sc, in); t && t->numel() == 1) {
                    std::vector<float> v;
                    if (t->to_f32(&v, err)) m->mag_scale = v[0];
                }
    }
    // graph order: STFT basis, normalisation filter, 15 encoder convs, decoder conv
    if (convs.size() != (size_t)(2 + kNBlk + 1)) {
        *err = path + ": expected " + std::to_string(2 + kNBlk + 1) + " Conv nodes in the 16 kHz branch, found " +
               std::to_string(convs.size());
        return false;
    }
    if (!read_conv(*convs[0], sc, &m->stft, err) || !read_conv(*convs[1], sc, &m->filt, err) ||
        !read_conv(*convs.back(), sc, &m->dec, err))
        return false;
    if (m->stft.out != 258 || m->stft.k != 256 || m->stft.stride != 64 || m->filt.k != 7 || m->dec.out != 1 || m->dec.in_g != 64) {
        *err = path + ": unexpected STFT / filter / decoder shapes";
        return false;
    }
    for (int i = 0; i < kNBlk; ++i) {
        if (!read_conv(*convs[2 + i], sc, &m->blk[i], err)) return false;
        const ConvW& c = m->blk[i];
        const Shape& s = kBlk[i];
        if (c.out != s.out || c.in_g != s.in_g || c.k != s.k || c.group != s.group || c.stride != s.stride ||
            (c.k == 5 && c.pad != 2)) {
            *err = path + ": encoder conv " + std::to_string(i) + " has an unexpected shape";
            return false;
        }
    }
    if (!lstm_if) { *err = path + ": no LSTM in the 16 kHz branch"; return false; }
    const onnx::Graph* with_state = branch(*lstm_if, "then_branch");  // the caller's h / c
    std::vector<const onnx::Graph*> sc2{&top, g16, with_state};
    int layer = 0;
    for (const onnx::Node& x : with_state->nodes) {
        if (x.op_type != "LSTM" || layer >= 2) continue;
        if (x.inputs.size() < 4) { *err = path + ": LSTM without bias"; return false; }
        m->lw[layer] = vals(sc2, x.inputs[1], err);
        m->lr[layer] = vals(sc2, x.inputs[2], err);
        m->lb[layer] = vals(sc2, x.inputs[3], err);
        if (m->lw[layer].size() != 256 * 64 || m->lr[layer].size() != 256 * 64 || m->lb[layer].size() != 512) {
            *err = path + ": LSTM layer " + std::to_string(layer) + " is not 64 units over 64 inputs";
            return false;
        }
        ++layer;
    }
    if (layer != 2) { *err = path + ": expected two LSTM layers"; return false; }
    if (m->pad_left != (float)kPadL || m->pad_right != (float)kPadL) { *err = path + ": unexpected STFT padding"; return false; }
    return true;
}

// ------------------------------------------------------------------ device layout
// one f32 blob; offsets (floats) of every tensor
struct Off {
    int64_t stft_w, filt_w, blk_w[kNBlk], blk_b[kNBlk], dec_w, dec_b, lw[2], lr[2], lb[2], total;
};

Off layout(const SileroHost& m) {
    Off o{};
    int64_t p = 0;
    auto take = [&](int64_t n) { const int64_t r = p; p += (n + 63) / 64 * 64; return r; };
    o.stft_w = take(258 * 256);
    o.filt_w = take(7);
    for (int i = 0; i < kNBlk; ++i) {
        o.blk_w[i] = take((int64_t)m.blk[i].w.size());
        o.blk_b[i] = take(m.blk[i].out);
    }
    o.dec_w = take(64);
    o.dec_b = take(1);
    for (int l = 0; l < 2; ++l) { o.lw[l] = take(256 * 64); o.lr[l] = take(256 * 64); o.lb[l] = take(256); }
    o.total = p;
    return o;
}

// ------------------------------------------------------------------ kernels

struct FrontArgs {
    const float* w;            // the weight blob
    Off o;
    float mag_scale;
    const float* pcm;          // [frames][480]
    float* feat;               // [frames][64]
};

// depthwise (k5, pad 2) + ReLU over C channels x T steps: dst[c][t]
__device__ void dw5(const float* __restrict__ w, const float* __restrict__ b, const float* src, float* dst, int C, int T) {
    for (int i = threadIdx.x; i < C * T; i += 256) {
        const int c = i / T, t = i - c * T;
        float s = b[c];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int u = t + j - 2;
            if (u >= 0 && u < T) s += w[c * 5 + j] * src[c * T + u];
        }
        dst[i] = fmaxf(s, 0.f);
    }
}
// 1x1 conv (stride s) Cin -> Cout: dst[o][t] = b[o] + sum_c w[o][c] src[c][t * s] (+ add[o][t]) (ReLU)
__device__ void pw(const float* __restrict__ w, const float* __restrict__ b, const float* src, int Cin, int Tin, int s,
                   float* dst, int Cout, int Tout, const float* add, bool relu) {
    for (int i = threadIdx.x; i < Cout * Tout; i += 256) {
        const int o = i / Tout, t = i - o * Tout;
        float acc = b[o];
        for (int c = 0; c < Cin; ++c) acc += w[o * Cin + c] * src[c * Tin + t * s];
        if (add) acc += add[i];
        dst[i] = relu ? fmaxf(acc, 0.f) : acc;
    }
}

// one workgroup per frame: everything before the LSTM
__global__ __launch_bounds__(256) void vad_front_kernel(FrontArgs a) {
    __shared__ float x[kPadded];
    __shared__ float ft[258 * kT];
    __shared__ float x1[258 * kT];
    __shared__ float d1[258 * kT];
    __shared__ float u[64 * kT], v[64 * kT], r[64 * kT];
    __shared__ float mean[kT], mm;
    const int f = blockIdx.x, tid = threadIdx.x;
    const float* in = a.pcm + (size_t)f * kVadFrame;
    for (int i = tid; i < kPadded; i += 256) {  // reflect padding (numpy / ONNX "reflect": the edge not repeated)
        int j = i - kPadL;
        if (j < 0) j = -j;
        if (j >= kVadFrame) j = 2 * (kVadFrame - 1) - j;
        x[i] = in[j];
    }
    __syncthreads();
    // STFT as a stride-64 convolution: ft[r][t] = basis[r] . x[64 t .. 64 t + 255]
    const float* basis = a.w + a.o.stft_w;
    for (int i = tid; i < 258 * kT; i += 256) {
        const int row = i / kT, t = i - row * kT;
        const float* bw = basis + (size_t)row * 256;
        const float* xs = x + 64 * t;
        float s = 0.f;
        for (int k = 0; k < 256; ++k) s += bw[k] * xs[k];
        ft[i] = s;
    }
    __syncthreads();
    // magnitude, log(1 + scale * magnitude) (graph: Pow 2, Add, Sqrt, Mul, Add 1, Log)
    for (int i = tid; i < 129 * kT; i += 256) {
        const float re = ft[i], im = ft[129 * kT + i];
        const float mg = sqrtf(re * re + im * im);
        x1[i] = mg;
        d1[i] = logf(a.mag_scale * mg + 1.0f);  // the spectrum, normalised below
    }
    __syncthreads();
    if (tid < kT) {  // mean over the 129 bins of each step
        float s = 0.f;
        for (int b = 0; b < 129; ++b) s += d1[b * kT + tid];
        mean[tid] = s / 129.0f;
    }
    __syncthreads();
    if (tid == 0) {  // reflect-pad 3, 7-tap smoothing, mean over the steps
        float ext[kT + 6];
        for (int i = 0; i < kT + 6; ++i) {
            int j = i - 3;
            if (j < 0) j = -j;
            if (j >= kT) j = 2 * (kT - 1) - j;
            ext[i] = mean[j];
        }
        const float* fw = a.w + a.o.filt_w;
        float tot = 0.f;
        for (int t = 0; t < kT; ++t) {
            float s = 0.f;
            for (int k = 0; k < 7; ++k) s += fw[k] * ext[t + k];
            tot += s;
        }
        mm = tot / kT;
    }
    __syncthreads();
    for (int i = tid; i < 129 * kT; i += 256) x1[129 * kT + i] = d1[i] - mm;  // [magnitude | normalised]
    __syncthreads();
    const float* W = a.w;
    const Off& o = a.o;
    // first_layer: dw(258) -> pw 258 -> 16, proj 258 -> 16 of x1, ReLU(sum)
    dw5(W + o.blk_w[0], W + o.blk_b[0], x1, d1, 258, kT);
    __syncthreads();
    pw(W + o.blk_w[2], W + o.blk_b[2], x1, 258, kT, 1, r, 16, kT, nullptr, false);
    __syncthreads();
    pw(W + o.blk_w[1], W + o.blk_b[1], d1, 258, kT, 1, u, 16, kT, r, true);
    __syncthreads();
    pw(W + o.blk_w[3], W + o.blk_b[3], u, 16, kT, 2, v, 16, 4, nullptr, true);            // 7 -> 4 steps
    __syncthreads();
    // encoder.3: dw(16) -> pw 16 -> 32, proj 16 -> 32
    dw5(W + o.blk_w[4], W + o.blk_b[4], v, d1, 16, 4);
    pw(W + o.blk_w[6], W + o.blk_b[6], v, 16, 4, 1, r, 32, 4, nullptr, false);
    __syncthreads();
    pw(W + o.blk_w[5], W + o.blk_b[5], d1, 16, 4, 1, u, 32, 4, r, true);
    __syncthreads();
    pw(W + o.blk_w[7], W + o.blk_b[7], u, 32, 4, 2, v, 32, 2, nullptr, true);             // 4 -> 2
    __syncthreads();
    // encoder.7: dw(32) -> pw 32 -> 32, identity residual
    dw5(W + o.blk_w[8], W + o.blk_b[8], v, d1, 32, 2);
    __syncthreads();
    pw(W + o.blk_w[9], W + o.blk_b[9], d1, 32, 2, 1, u, 32, 2, v, true);
    __syncthreads();
    pw(W + o.blk_w[10], W + o.blk_b[10], u, 32, 2, 2, v, 32, 1, nullptr, true);           // 2 -> 1
    __syncthreads();
    // encoder.11: dw(32) -> pw 32 -> 64, proj 32 -> 64
    dw5(W + o.blk_w[11], W + o.blk_b[11], v, d1, 32, 1);
    pw(W + o.blk_w[13], W + o.blk_b[13], v, 32, 1, 1, r, 64, 1, nullptr, false);
    __syncthreads();
    pw(W + o.blk_w[12], W + o.blk_b[12], d1, 32, 1, 1, u, 64, 1, r, true);
    __syncthreads();
    pw(W + o.blk_w[14], W + o.blk_b[14], u, 64, 1, 1, a.feat + (size_t)f * 64, 64, 1, nullptr, true);
}

struct LstmArgs {
    const float* w;
    Off o;
    const float* feat;   // [frames][64]
    int n;
    float* state;        // h [2][64], c [2][64]: in and out
    float* prob;         // [frames]
};

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + expf(-z)); }

// The recurrence over the frames: threads 0-255 own layer 1's gate rows, 256-511 layer 2's; layer 2
// works on frame s - 1 while layer 1 works on frame s.  ONNX gate rows: i, o, f, c (64 each).
__global__ __launch_bounds__(512) void vad_lstm_kernel(LstmArgs a) {
    __shared__ float h[2][64], c[2][64], z[2][256], xin[2][64];
    const int tid = threadIdx.x, L = tid >> 8, row = tid & 255;
    float wr[64], rr[64];
    const float* W = a.w + a.o.lw[L] + (size_t)row * 64;
    const float* R = a.w + a.o.lr[L] + (size_t)row * 64;
#pragma unroll
    for (int k = 0; k < 64; ++k) { wr[k] = W[k]; rr[k] = R[k]; }
    const float bias = a.w[a.o.lb[L] + row];  // B_w + B_r, summed at load
    if (tid < 128) { h[tid >> 6][tid & 63] = a.state[tid]; c[tid >> 6][tid & 63] = a.state[128 + tid]; }
    if (tid < 64) xin[0][tid] = a.n > 0 ? a.feat[tid] : 0.f;
    const float dw = tid >= 256 && tid < 320 ? a.w[a.o.dec_w + (tid - 256)] : 0.f;
    const float db = a.w[a.o.dec_b];
    __syncthreads();
    for (int s = 0; s <= a.n; ++s) {
        const int cur = s & 1;
        const bool act = L == 0 ? s < a.n : s >= 1;
        if (act) {
            const float* x = L == 0 ? xin[cur] : h[0];  // layer 2's input: layer 1's h of frame s - 1
            float acc = bias;
#pragma unroll
            for (int k = 0; k < 64; ++k) acc += wr[k] * x[k];
#pragma unroll
            for (int k = 0; k < 64; ++k) acc += rr[k] * h[L][k];
            z[L][row] = acc;
        }
        if (tid >= 448 && s + 1 < a.n) xin[cur ^ 1][tid - 448] = a.feat[(size_t)(s + 1) * 64 + tid - 448];
        __syncthreads();
        if ((tid < 64 && s < a.n) || (tid >= 256 && tid < 320 && s >= 1)) {
            const int u = tid & 63;
            const float ig = sigm(z[L][u]), og = sigm(z[L][64 + u]), fg = sigm(z[L][128 + u]);
            const float gg = tanhf(z[L][192 + u]);
            const float cn = fg * c[L][u] + ig * gg;
            const float hn = og * tanhf(cn);
            c[L][u] = cn;
            h[L][u] = hn;
            if (L == 1) {  // ReLU -> 1x1 conv -> sigmoid: the frame's speech probability
                const float t = wave_sum(fmaxf(hn, 0.f) * dw);
                if (u == 0) a.prob[s - 1] = sigm(t + db);
            }
        }
        __syncthreads();
    }
    if (tid < 128) { a.state[tid] = h[tid >> 6][tid & 63]; a.state[128 + tid] = c[tid >> 6][tid & 63]; }
}

}  // namespace

struct VadEngine::Ptrs {
    Off o;
    float mag_scale;
};

VadEngine::VadEngine(const std::string& model_path, int device) : dev_(device) {
    SileroHost m;
    std::string err;
    if (!load_silero(model_path, &m, &err)) throw std::runtime_error(err);
    p_ = new Ptrs{layout(m), m.mag_scale};
    std::vector<float> blob((size_t)p_->o.total, 0.f);
    auto put = [&](int64_t off, const std::vector<float>& v) { std::copy(v.begin(), v.end(), blob.begin() + off); };
    put(p_->o.stft_w, m.stft.w);
    put(p_->o.filt_w, m.filt.w);
    for (int i = 0; i < kNBlk; ++i) { put(p_->o.blk_w[i], m.blk[i].w); put(p_->o.blk_b[i], m.blk[i].b); }
    put(p_->o.dec_w, m.dec.w);
    put(p_->o.dec_b, m.dec.b);
    for (int l = 0; l < 2; ++l) {
        put(p_->o.lw[l], m.lw[l]);
        put(p_->o.lr[l], m.lr[l]);
        std::vector<float> b(256);
        for (int i = 0; i < 256; ++i) b[i] = m.lb[l][i] + m.lb[l][256 + i];
        put(p_->o.lb[l], b);
    }
    select();
    HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipMalloc(&wbuf_, blob.size() * 4));
    HIP_CHECK(hipMemcpy(wbuf_, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMalloc(&state_, 256 * 4));
    reset_state();
}

VadEngine::~VadEngine() {  // teardown errors are not reportable from a destructor
    (void)hipSetDevice(dev_);
    if (st_) (void)hipStreamSynchronize(st_);
    for (void* p : {(void*)wbuf_, (void*)state_, (void*)pcm_, (void*)feat_, (void*)prob_})
        if (p) (void)hipFree(p);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    if (st_) (void)hipStreamDestroy(st_);
    delete p_;
}

void VadEngine::select() const { HIP_CHECK(hipSetDevice(dev_)); }

void VadEngine::reset_state() {
    select();
    HIP_CHECK(hipMemset(state_, 0, 256 * 4));
}

void VadEngine::ensure(int n) {
    if (n <= cap_frames_) return;
    for (void* p : {(void*)pcm_, (void*)feat_, (void*)prob_})
        if (p) HIP_CHECK(hipFree(p));
    const int cap = std::max(n, 1024);
    HIP_CHECK(hipMalloc(&pcm_, (size_t)cap * kVadFrame * 4));
    HIP_CHECK(hipMalloc(&feat_, (size_t)cap * 64 * 4));
    HIP_CHECK(hipMalloc(&prob_, (size_t)cap * 4));
    cap_frames_ = cap;
}

void VadEngine::probs(const float* pcm_host, int n, float* probs_host) {
    if (n <= 0) return;
    select();
    ensure(n);
    HIP_CHECK(hipMemcpyAsync(pcm_, pcm_host, (size_t)n * kVadFrame * 4, hipMemcpyHostToDevice, st_));
    HIP_CHECK(hipEventRecord(ev_[0], st_));
    FrontArgs fa{(const float*)wbuf_, p_->o, p_->mag_scale, pcm_, feat_};
    hipLaunchKernelGGL(vad_front_kernel, dim3(n), dim3(256), 0, st_, fa);
    SPT_LAUNCH_CHECK();
    LstmArgs la{(const float*)wbuf_, p_->o, feat_, n, state_, prob_};
    hipLaunchKernelGGL(vad_lstm_kernel, dim3(1), dim3(512), 0, st_, la);
    SPT_LAUNCH_CHECK();
    HIP_CHECK(hipEventRecord(ev_[1], st_));
    HIP_CHECK(hipMemcpyAsync(probs_host, prob_, (size_t)n * 4, hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
    last_ms_ = ms;
}

// ------------------------------------------------------------------ SmoothedVad (host)
void SmoothedVad::buffer(const float* frame, int n) {
    buf_.emplace_back(frame, frame + n);
    while ((int)buf_.size() > prefill_ + 1) buf_.erase(buf_.begin());
}

int SmoothedVad::push(const float* frame, int n, bool voice, std::vector<float>* out) {
    buffer(frame, n);  // 1. every frame is buffered for the pre-roll
    if (!in_speech_ && voice) {  // potential start: onset frames
        if (++ons_ >= onset_) {
            in_speech_ = true;
            hang_ = hangover_;
            ons_ = 0;
            for (const auto& b : buf_) out->insert(out->end(), b.begin(), b.end());
            return 2;
        }
        return 0;
    }
    if (in_speech_ && voice) {
        hang_ = hangover_;
        out->insert(out->end(), frame, frame + n);
        return 1;
    }
    if (in_speech_ && !voice) {
        if (hang_ > 0) {
            --hang_;
            out->insert(out->end(), frame, frame + n);
            return 1;
        }
        in_speech_ = false;
        return 0;
    }
    ons_ = 0;  // silence or a broken onset
    return 0;
}

void SmoothedVad::push_unchecked(const float* frame, int n, std::vector<float>* out) {
    buffer(frame, n);
    out->insert(out->end(), frame, frame + n);
}

void SmoothedVad::reset() {
    buf_.clear();
    hang_ = 0;
    ons_ = 0;
    in_speech_ = false;
}

}  // namespace spt
