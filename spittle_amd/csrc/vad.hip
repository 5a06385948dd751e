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
#include "vad_model.h"

namespace spt {

constexpr int kPadded = kVadFrame + 2 * kPadL;  // 672
constexpr int kT = 7;          // STFT steps: (672 - 256) / 64 + 1

// ------------------------------------------------------------------ kernels
namespace {

struct FrontArgs {
    const float* w;            // the weight blob
    SileroOff o;
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
    const SileroOff& o = a.o;
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
    SileroOff o;
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
    SileroOff o;
    float mag_scale;
};

VadEngine::VadEngine(const std::string& model_path, int device) : dev_(device) {
    SileroHost m;
    std::string err;
    if (!load_silero(model_path, &m, &err)) throw std::runtime_error(err);
    p_ = new Ptrs{SileroOff{}, m.mag_scale};
    const std::vector<float> blob = silero_blob(m, &p_->o);
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
    // freed and cleared first: if an allocation below throws, the destructor finds no stale pointer
    for (void* p : {(void*)pcm_, (void*)feat_, (void*)prob_})
        if (p) HIP_CHECK(hipFree(p));
    pcm_ = nullptr;
    feat_ = nullptr;
    prob_ = nullptr;
    cap_frames_ = 0;
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
