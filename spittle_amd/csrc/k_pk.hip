// k_pk.hip -- Parakeet-V3 (FastConformer-TDT) kernels: front end, subsampling, rel-pos
// attention, convolution module and the TDT greedy step.  Replaces the ONNX Runtime graph
// transcribe-rs' ParakeetEngine runs (/root/reference/src-tauri/src/managers/transcription.rs:
// 278-297 load, 505-513 transcribe_samples); the model is NeMo's (oracle/parakeet_oracle.h).
//
// The dense products (DFT, pointwise convolutions, linear layers, the joint's encoder
// projection) are MFMA GEMMs (k_gemm.hip); what is here is the memory-bound glue, each kernel
// one pass over its tensor.  Activations are [rows][channels] with channels contiguous, so
// every kernel's lanes walk the channel axis (coalesced); the frame axis carries the masks.
#include "common.h"
#include "kernels.h"
#include "pk_kernels.h"

#include <algorithm>

namespace spt {

namespace {

inline int grid_of(int64_t n, int tpb = 256) {
    int64_t g = (n + tpb - 1) / tpb;
    return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

template <typename T> __device__ __forceinline__ T* tp(void* p) { return (T*)p; }
template <typename T> __device__ __forceinline__ const T* tp(const void* p) { return (const T*)p; }

// ---------------------------------------------------------------- front end
__global__ __launch_bounds__(256) void frames_kernel(const float* __restrict__ pcm, int64_t stride,
                                                     const int* __restrict__ nsamp, int Tp,
                                                     const float* __restrict__ win, float* __restrict__ frames) {
    const int t = blockIdx.x, b = blockIdx.y;
    const int n = nsamp[b];
    const float* x = pcm + (size_t)b * stride;
    float* row = frames + ((size_t)b * Tp + t) * PK_NFFT;
    for (int i = threadIdx.x; i < PK_NFFT; i += 256) {
        const int s = t * PK_HOP + i - PK_NFFT / 2;  // centre padding: n_fft / 2 zeros each side
        float v = 0.0f;
        if (s >= 0 && s < n) v = x[s] - (s > 0 ? __fmul_rn(0.97f, x[s - 1]) : 0.0f);  // pre-emphasis
        row[i] = __fmul_rn(v, win[i]);
    }
}

// one workgroup per frame: |X_k|^2 -> mel filterbank (fbT [257][n_mels]) -> log(x + 2^-24)
__global__ __launch_bounds__(128) void melpow_kernel(const float* __restrict__ spec, const float* __restrict__ fbT,
                                                     int n_mels, float* __restrict__ mel) {
    __shared__ float pw[PK_NBIN];
    const size_t r = blockIdx.x;
    const float* s = spec + r * PK_DFT_N;
    for (int k = threadIdx.x; k < PK_NBIN; k += 128) {
        const float re = s[k], im = s[PK_NBIN + k];
        pw[k] = re * re + im * im;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n_mels; j += 128) {
        float acc = 0.0f;
        for (int k = 0; k < PK_NBIN; ++k) acc += fbT[k * n_mels + j] * pw[k];
        mel[r * n_mels + j] = logf(acc + 5.9604644775390625e-08f);
    }
}

// per (utterance, 32 mel bands): 8 frame groups x 32 bands, f64 sums; three passes
__global__ __launch_bounds__(256) void mel_norm_kernel(float* __restrict__ mel, const int* __restrict__ lens, int Tp,
                                                       int n_mels) {
    __shared__ double red[8][33];
    const int b = blockIdx.x, jl = threadIdx.x & 31, tg = threadIdx.x >> 5;
    const int j = blockIdx.y * 32 + jl;
    const int T = lens[b * 4];
    float* base = mel + (size_t)b * Tp * n_mels;
    const bool ok = j < n_mels;
    double s = 0;
    if (ok)
        for (int t = tg; t < T; t += 8) s += base[(size_t)t * n_mels + j];
    red[tg][jl] = s;
    __syncthreads();
    double mean = 0;
    for (int g = 0; g < 8; ++g) mean += red[g][jl];
    mean /= T;
    __syncthreads();
    double v = 0;
    if (ok)
        for (int t = tg; t < T; t += 8) {
            const double e = base[(size_t)t * n_mels + j] - mean;
            v += e * e;
        }
    red[tg][jl] = v;
    __syncthreads();
    double var = 0;
    for (int g = 0; g < 8; ++g) var += red[g][jl];
    const double sd = sqrt(var / (T > 1 ? T - 1 : 1)) + 1e-5;
    if (!ok) return;
    for (int t = tg; t < Tp; t += 8) {
        float* p = base + (size_t)t * n_mels + j;
        *p = t < T ? (float)((*p - mean) / sd) : 0.0f;
    }
}

// ---------------------------------------------------------------- subsampling
template <typename T>
__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ mel, const int* __restrict__ lens,
                                                    int B, int Tp, int F, const float* __restrict__ w,
                                                    const float* __restrict__ bias, int C, T* __restrict__ y, int T1p,
                                                    int F1) {
    const int64_t total = (int64_t)B * T1p * F1 * C;
    for (int64_t idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int c = (int)(idx % C);
        int64_t q = idx / C;
        const int f = (int)(q % F1);
        q /= F1;
        const int t = (int)(q % T1p);
        const int b = (int)(q / T1p);
        const int Tb = min(lens[b * 4], Tp);
        float acc = bias[c];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int tt = 2 * t - 1 + i;
            if (tt < 0 || tt >= Tb) continue;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ff = 2 * f - 1 + j;
                if (ff >= 0 && ff < F) acc += w[c * 9 + i * 3 + j] * mel[((size_t)b * Tp + tt) * F + ff];
            }
        }
        y[idx] = from_f<T>(fmaxf(acc, 0.0f));
    }
}

template <typename T>
__global__ __launch_bounds__(256) void dwconv_kernel(const T* __restrict__ x, const int* __restrict__ lens, int stage,
                                                     int B, int Tip, int Fi, const float* __restrict__ w,
                                                     const float* __restrict__ bias, int C, T* __restrict__ y, int Top,
                                                     int Fo) {
    const int64_t total = (int64_t)B * Top * Fo * C;
    for (int64_t idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int c = (int)(idx % C);
        int64_t q = idx / C;
        const int f = (int)(q % Fo);
        q /= Fo;
        const int t = (int)(q % Top);
        const int b = (int)(q / Top);
        const int Tb = min(lens[b * 4 + stage], Tip);
        float acc = bias[c];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int tt = 2 * t - 1 + i;
            if (tt < 0 || tt >= Tb) continue;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ff = 2 * f - 1 + j;
                if (ff >= 0 && ff < Fi) acc += w[c * 9 + i * 3 + j] * to_f<T>(x[(((size_t)b * Tip + tt) * Fi + ff) * C + c]);
            }
        }
        y[idx] = from_f<T>(acc);
    }
}

template <typename T>
__global__ void relpos_kernel(int Tp, int d, T* __restrict__ pe) {
    const int64_t total = (int64_t)(2 * Tp - 1) * (d / 2);
    for (int64_t idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int k = (int)(idx % (d / 2));
        const int r = (int)(idx / (d / 2));
        const double pos = (double)(Tp - 1 - r);
        const double div = exp(-(2.0 * k) * log(10000.0) / d);
        pe[(size_t)r * d + 2 * k] = from_f<T>((float)sin(pos * div));
        pe[(size_t)r * d + 2 * k + 1] = from_f<T>((float)cos(pos * div));
    }
}

// ---------------------------------------------------------------- rel-pos attention
// One wave per (query, head, utterance).  Scores for 64 keys at a time (a lane per key, its
// k row and p row read as 16-byte vectors), kept in LDS; exact softmax; P.V with lanes over
// the head dimension.  ac = (q + u) . k_j, bd = (q + v) . p_{Tp-1-i+j} (NeMo's rel_shift as an
// index), scores / sqrt(dk).
template <typename T> __device__ __forceinline__ void ld8(const T* p, float* o);
template <> __device__ __forceinline__ void ld8<float>(const float* p, float* o) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <> __device__ __forceinline__ void ld8<f16>(const f16* p, float* o) {
    const f16x8 v = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
}
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, float* o) {
    const uint4 v = *(const uint4*)p;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = bf2f((bf16)(w[i] & 0xffff));
        o[2 * i + 1] = bf2f((bf16)(w[i] >> 16));
    }
}

template <typename T>
__global__ __launch_bounds__(64) void rel_attn_kernel(const T* __restrict__ qkv, const T* __restrict__ p, int ldp,
                                                      const float* __restrict__ pu, const float* __restrict__ pv,
                                                      const int* __restrict__ lens, int Tp, int H, int dk,
                                                      T* __restrict__ out) {
    extern __shared__ float sm[];  // qu[dk] | qv[dk] | scores[Tp]
    float* qu = sm;
    float* qv = sm + dk;
    float* sc = sm + 2 * dk;
    const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z, lane = threadIdx.x;
    const int d = H * dk;
    const int T3 = lens[b * 4 + 3];
    T* orow = out + ((size_t)b * Tp + i) * d + h * dk;
    if (i >= T3) {
        for (int e = lane; e < dk; e += 64) orow[e] = from_f<T>(0.0f);
        return;
    }
    const T* base = qkv + (size_t)b * Tp * 3 * d;
    for (int e = lane; e < dk; e += 64) {
        const float q = to_f<T>(base[(size_t)i * 3 * d + h * dk + e]);
        qu[e] = q + pu[h * dk + e];
        qv[e] = q + pv[h * dk + e];
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)dk);
    float mx = -INFINITY;
    for (int j0 = 0; j0 < T3; j0 += 64) {
        const int j = j0 + lane;
        if (j < T3) {
            const T* kr = base + (size_t)j * 3 * d + d + h * dk;
            const T* pr = p + (size_t)(Tp - 1 - i + j) * ldp + h * dk;
            float ac = 0.0f, bd = 0.0f;
            for (int e = 0; e < dk; e += 8) {
                float kv[8], pv8[8];
                ld8<T>(kr + e, kv);
                ld8<T>(pr + e, pv8);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    ac += qu[e + u] * kv[u];
                    bd += qv[e + u] * pv8[u];
                }
            }
            const float s = (ac + bd) * scale;
            sc[j] = s;
            mx = fmaxf(mx, s);
        }
    }
    mx = wave_max(mx);
    float l = 0.0f;
    for (int j = lane; j < T3; j += 64) {
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        l += e;
    }
    l = wave_sum(l);
    __syncthreads();
    for (int e = lane; e < dk; e += 64) {
        float acc = 0.0f;
        const T* vc = base + 2 * d + h * dk + e;
        for (int j = 0; j < T3; ++j) acc += sc[j] * to_f<T>(vc[(size_t)j * 3 * d]);
        orow[e] = from_f<T>(acc / l);
    }
}

// ---------------------------------------------------------------- convolution module
template <typename T>
__global__ __launch_bounds__(256) void conv_module_kernel(const T* __restrict__ a, const int* __restrict__ lens, int B,
                                                          int Tp, int d, int K, const float* __restrict__ dw_w,
                                                          const float* __restrict__ dw_b, const float* __restrict__ bn_g,
                                                          const float* __restrict__ bn_b, const float* __restrict__ bn_m,
                                                          const float* __restrict__ bn_v, T* __restrict__ out) {
    const int64_t total = (int64_t)B * Tp * d;
    for (int64_t idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int i = (int)(idx % d);
        const int64_t row = idx / d;
        const int t = (int)(row % Tp), b = (int)(row / Tp);
        const int T3 = lens[b * 4 + 3];
        if (t >= T3) { out[idx] = from_f<T>(0.0f); continue; }
        const float bs = bn_g[i] / sqrtf(bn_v[i] + 1e-5f), bt = bn_b[i] - bn_m[i] * bs;
        float acc = dw_b[i];
        for (int j = 0; j < K; ++j) {
            const int tt = t - K / 2 + j;
            if (tt < 0 || tt >= T3) continue;
            const T* ar = a + ((size_t)b * Tp + tt) * 2 * d;
            const float g = to_f<T>(ar[i]) * (1.0f / (1.0f + expf(-to_f<T>(ar[d + i]))));  // GLU
            acc += dw_w[i * K + j] * g;
        }
        const float z = acc * bs + bt;
        out[idx] = from_f<T>(z / (1.0f + expf(-z)));  // Swish
    }
}

// ---------------------------------------------------------------- weight placement
template <typename T>
__global__ void place_copy_kernel(const float* __restrict__ s, int64_t n, T* __restrict__ d) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = from_f<T>(s[i]);
}
__global__ void place_transpose_kernel(const float* __restrict__ s, int N, int K, float* __restrict__ d, int ld,
                                       int row0) {
    const int64_t total = (int64_t)N * K;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int n = (int)(i % N), k = (int)(i / N);  // n fastest: coalesced writes
        d[(size_t)(row0 + k) * ld + n] = s[(size_t)n * K + k];
    }
}
template <typename T>
__global__ void place_subperm_kernel(const float* __restrict__ s, int N, int C, int F, T* __restrict__ d) {
    const int64_t total = (int64_t)N * C * F;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i % C);
        const int64_t q = i / C;
        const int f = (int)(q % F);
        const int64_t n = q / F;
        d[i] = from_f<T>(s[(n * C + c) * F + f]);  // dst [n][f * C + c] <- src [n][c * F + f]
    }
}

// ---------------------------------------------------------------- TDT greedy step
// y[b][n] partial over a K slab: lanes over n (W^T rows are contiguous in n), the slab's x
// rows for every utterance staged in LDS as [k][BM] (one ds_read_b128 feeds four rows).
template <int XM, int BM>
__global__ __launch_bounds__(256) void gemv_t_kernel(PkGemvArgs a) {
    extern __shared__ float xs[];  // [KC][BM]
    const int KC = a.K / a.ksplit, s = blockIdx.y, k0 = s * KC;
    const int P = a.P, B = a.B;
    for (int idx = threadIdx.x; idx < KC * BM; idx += 256) {
        const int k = idx % KC, b = idx / KC, kk = k0 + k;
        float v = 0.0f;
        if (b < B) {
            if constexpr (XM == PKX_LSTM0) {
                v = kk < P ? a.emb[(size_t)a.st[b].tok * P + kk] : a.h0[(size_t)b * P + kk - P];
            } else if constexpr (XM == PKX_LSTM1) {
                v = kk < P ? a.h0[(size_t)b * P + kk] : a.h1[(size_t)b * P + kk - P];
            } else if constexpr (XM == PKX_PRED) {
                v = a.h1[(size_t)b * P + kk];
            } else {
                const PkState sb = a.st[b];
                float g;
                if (sb.upd) {
                    g = a.pred_b[kk];
                    for (int q = 0; q < a.pred_split; ++q) g += a.pred_part[((size_t)q * B + b) * a.pred_Npad + kk];
                    if (blockIdx.x == 0) a.gp[(size_t)b * P + kk] = g;
                } else {
                    g = a.gp[(size_t)b * P + kk];
                }
                const int t = min(sb.t, a.T3p - 1);
                v = fmaxf(a.fe[((size_t)b * a.T3p + t) * P + kk] + g, 0.0f);  // ReLU(enc + pred)
            }
        }
        xs[k * BM + b] = v;
    }
    __syncthreads();
    const int n = blockIdx.x * 256 + threadIdx.x;
    float acc[BM];
#pragma unroll
    for (int b = 0; b < BM; ++b) acc[b] = 0.0f;
    const float* w = a.WT + (size_t)k0 * a.Npad + n;
#pragma unroll 4
    for (int k = 0; k < KC; ++k) {
        const float wv = w[(size_t)k * a.Npad];
#pragma unroll
        for (int b = 0; b < BM; b += 4) {
            const float4 x4 = *(const float4*)&xs[k * BM + b];
            acc[b] += wv * x4.x;
            acc[b + 1] += wv * x4.y;
            acc[b + 2] += wv * x4.z;
            acc[b + 3] += wv * x4.w;
        }
    }
#pragma unroll
    for (int b = 0; b < BM; ++b)
        if (b < B) a.part[((size_t)s * B + b) * a.Npad + n] = acc[b];
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_cell_kernel(const float* __restrict__ part, int ksplit, int Npad,
                                                        const float* __restrict__ b_ih, const float* __restrict__ b_hh,
                                                        int B, int P, const PkState* __restrict__ st,
                                                        float* __restrict__ h, float* __restrict__ c) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= B * P) return;
    const int b = idx / P, j = idx - b * P;
    if (!st[b].upd) return;
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int n = q * P + j;
        float v = b_ih[n] + b_hh[n];
        for (int s = 0; s < ksplit; ++s) v += part[((size_t)s * B + b) * Npad + n];
        g[q] = v;
    }
    const float ig = sigm(g[0]), fg = sigm(g[1]), gg = tanhf(g[2]), og = sigm(g[3]);
    const float cn = fg * c[idx] + ig * gg;
    c[idx] = cn;
    h[idx] = og * tanhf(cn);
}

// one workgroup per utterance: joint logits (slab sums + bias), token top-2 and duration
// argmax (first maximum wins, as the oracle's strict >), then the TDT bookkeeping
__global__ __launch_bounds__(256) void joint_fin_kernel(PkFinArgs a) {
    __shared__ float s1[256], s2[256], sd[256];
    __shared__ int i1[256], id_[256];
    const int b = blockIdx.x, tid = threadIdx.x;
    PkState* sb = a.st + b;
    if (sb->done) return;  // uniform
    const int V = a.V, NO = V + 1 + a.n_dur;
    float b1 = -INFINITY, b2 = -INFINITY, bdv = -INFINITY;
    int t1 = 0x7fffffff, td = 0x7fffffff;
    for (int n = tid; n < NO; n += 256) {
        float v = a.bias[n];
        for (int s = 0; s < a.ksplit; ++s) v += a.part[((size_t)s * a.B + b) * a.Npad + n];
        if (n <= V) {
            if (v > b1) { b2 = b1; b1 = v; t1 = n; }
            else if (v > b2) b2 = v;
        } else if (v > bdv) { bdv = v; td = n - V - 1; }
    }
    s1[tid] = b1; s2[tid] = b2; i1[tid] = t1; sd[tid] = bdv; id_[tid] = td;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            const float a1 = s1[tid], a2 = s2[tid], c1 = s1[tid + o], c2 = s2[tid + o];
            const int ai = i1[tid], ci = i1[tid + o];
            const bool take = c1 > a1 || (c1 == a1 && ci < ai);
            s1[tid] = take ? c1 : a1;
            i1[tid] = take ? ci : ai;
            s2[tid] = fmaxf(fmaxf(a2, c2), take ? a1 : c1);
            const float e1 = sd[tid], e2 = sd[tid + o];
            const int ei = id_[tid], ej = id_[tid + o];
            if (e2 > e1 || (e2 == e1 && ej < ei)) { sd[tid] = e2; id_[tid] = ej; }
        }
        __syncthreads();
    }
    if (tid != 0) return;
    PkState s = *sb;
    const int tk = i1[0];
    int skip = id_[0];
    if (tk != V) {
        if (s.n_out < a.cap) {
            const size_t o = (size_t)b * a.cap + s.n_out;
            a.out_tok[o] = tk;
            a.out_frame[o] = s.t;
            a.out_t1[o] = s1[0];
            a.out_t2[o] = s2[0];
        }
        s.n_out++;
        s.upd = 1;
        s.tok = tk;
        s.at_t++;
    } else {
        s.upd = 0;
    }
    if (skip == 0 && (tk == V || s.at_t >= a.max_symbols)) skip = 1;
    if (skip > 0) s.at_t = 0;
    s.t += skip;
    if (s.t >= a.lens[b * 4 + 3]) s.done = 1;
    *sb = s;
}

__global__ void state_init_kernel(PkState* st, int B, int V, float* h, float* c, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < B) st[i] = PkState{0, 0, 0, 0, 1, V};
    if (i < n) { h[i] = 0.0f; c[i] = 0.0f; }
}

}  // namespace

void pk_frames(const float* pcm, int64_t stride, const int* nsamp, int B, int Tp, const float* window, float* frames,
               hipStream_t st) {
    hipLaunchKernelGGL(frames_kernel, dim3(Tp, B), dim3(256), 0, st, pcm, stride, nsamp, Tp, window, frames);
    SPT_LAUNCH_CHECK();
}

void pk_melpow(const float* spec, int M, const float* fbT, int n_mels, float* mel, hipStream_t st) {
    hipLaunchKernelGGL(melpow_kernel, dim3(M), dim3(128), 0, st, spec, fbT, n_mels, mel);
    SPT_LAUNCH_CHECK();
}

void pk_mel_norm(float* mel, const int* lens, int B, int Tp, int n_mels, hipStream_t st) {
    hipLaunchKernelGGL(mel_norm_kernel, dim3(B, cdiv(n_mels, 32)), dim3(256), 0, st, mel, lens, Tp, n_mels);
    SPT_LAUNCH_CHECK();
}

void pk_conv0(int dtype, const float* mel, const int* lens, int B, int Tp, int F, const float* w, const float* bias,
              int C, void* y, int T1p, int F1, hipStream_t st) {
    const int g = grid_of((int64_t)B * T1p * F1 * C);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(conv0_kernel<f16>, dim3(g), dim3(256), 0, st, mel, lens, B, Tp, F, w, bias, C, (f16*)y, T1p, F1);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(conv0_kernel<bf16>, dim3(g), dim3(256), 0, st, mel, lens, B, Tp, F, w, bias, C, (bf16*)y, T1p, F1);
    else
        hipLaunchKernelGGL(conv0_kernel<float>, dim3(g), dim3(256), 0, st, mel, lens, B, Tp, F, w, bias, C, (float*)y, T1p, F1);
    SPT_LAUNCH_CHECK();
}

void pk_dwconv(int dtype, const void* x, const int* lens, int stage, int B, int Tip, int Fi, const float* w,
               const float* bias, int C, void* y, int Top, int Fo, hipStream_t st) {
    const int g = grid_of((int64_t)B * Top * Fo * C);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(dwconv_kernel<f16>, dim3(g), dim3(256), 0, st, (const f16*)x, lens, stage, B, Tip, Fi, w, bias,
                           C, (f16*)y, Top, Fo);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(dwconv_kernel<bf16>, dim3(g), dim3(256), 0, st, (const bf16*)x, lens, stage, B, Tip, Fi, w,
                           bias, C, (bf16*)y, Top, Fo);
    else
        hipLaunchKernelGGL(dwconv_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, lens, stage, B, Tip, Fi, w,
                           bias, C, (float*)y, Top, Fo);
    SPT_LAUNCH_CHECK();
}

void pk_relpos(int dtype, int Tp, int d, void* pe, hipStream_t st) {
    const int g = grid_of((int64_t)(2 * Tp - 1) * (d / 2));
    if (dtype == DT_F16) hipLaunchKernelGGL(relpos_kernel<f16>, dim3(g), dim3(256), 0, st, Tp, d, (f16*)pe);
    else if (dtype == DT_BF16) hipLaunchKernelGGL(relpos_kernel<bf16>, dim3(g), dim3(256), 0, st, Tp, d, (bf16*)pe);
    else hipLaunchKernelGGL(relpos_kernel<float>, dim3(g), dim3(256), 0, st, Tp, d, (float*)pe);
    SPT_LAUNCH_CHECK();
}

void pk_rel_attn(int dtype, const void* qkv, const void* p, int ldp, const float* pu, const float* pv, const int* lens,
                 int B, int Tp, int H, int dk, void* out, hipStream_t st) {
    if (dk % 8 || dk > 256) throw std::runtime_error("pk_rel_attn: head dim must be a multiple of 8, <= 256");
    const size_t smem = (size_t)(2 * dk + Tp) * 4;
    if (smem > 64 * 1024) throw std::runtime_error("pk_rel_attn: too many frames for the LDS score row");
    dim3 grid(Tp, H, B);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(rel_attn_kernel<f16>, grid, dim3(64), smem, st, (const f16*)qkv, (const f16*)p, ldp, pu, pv,
                           lens, Tp, H, dk, (f16*)out);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(rel_attn_kernel<bf16>, grid, dim3(64), smem, st, (const bf16*)qkv, (const bf16*)p, ldp, pu, pv,
                           lens, Tp, H, dk, (bf16*)out);
    else
        hipLaunchKernelGGL(rel_attn_kernel<float>, grid, dim3(64), smem, st, (const float*)qkv, (const float*)p, ldp, pu,
                           pv, lens, Tp, H, dk, (float*)out);
    SPT_LAUNCH_CHECK();
}

void pk_conv_module(int dtype, const void* a, const int* lens, int B, int Tp, int d, int K, const float* dw_w,
                    const float* dw_b, const float* bn_g, const float* bn_b, const float* bn_m, const float* bn_v,
                    void* out, hipStream_t st) {
    const int g = grid_of((int64_t)B * Tp * d);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(conv_module_kernel<f16>, dim3(g), dim3(256), 0, st, (const f16*)a, lens, B, Tp, d, K, dw_w,
                           dw_b, bn_g, bn_b, bn_m, bn_v, (f16*)out);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(conv_module_kernel<bf16>, dim3(g), dim3(256), 0, st, (const bf16*)a, lens, B, Tp, d, K, dw_w,
                           dw_b, bn_g, bn_b, bn_m, bn_v, (bf16*)out);
    else
        hipLaunchKernelGGL(conv_module_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)a, lens, B, Tp, d, K,
                           dw_w, dw_b, bn_g, bn_b, bn_m, bn_v, (float*)out);
    SPT_LAUNCH_CHECK();
}

void pk_place(int mode, int dtype, const float* src, int N, int K, void* dst, int ld, int row0, int C, int F,
              hipStream_t st) {
    if (mode == PK_PLACE_TRANSPOSE) {
        hipLaunchKernelGGL(place_transpose_kernel, dim3(grid_of((int64_t)N * K)), dim3(256), 0, st, src, N, K,
                           (float*)dst, ld, row0);
    } else if (mode == PK_PLACE_SUBPERM) {
        const int g = grid_of((int64_t)N * C * F);
        if (dtype == DT_F16) hipLaunchKernelGGL(place_subperm_kernel<f16>, dim3(g), dim3(256), 0, st, src, N, C, F, (f16*)dst);
        else if (dtype == DT_BF16)
            hipLaunchKernelGGL(place_subperm_kernel<bf16>, dim3(g), dim3(256), 0, st, src, N, C, F, (bf16*)dst);
        else hipLaunchKernelGGL(place_subperm_kernel<float>, dim3(g), dim3(256), 0, st, src, N, C, F, (float*)dst);
    } else {
        const int64_t n = (int64_t)N * K;
        const int g = grid_of(n);
        if (dtype == DT_F16) hipLaunchKernelGGL(place_copy_kernel<f16>, dim3(g), dim3(256), 0, st, src, n, (f16*)dst);
        else if (dtype == DT_BF16) hipLaunchKernelGGL(place_copy_kernel<bf16>, dim3(g), dim3(256), 0, st, src, n, (bf16*)dst);
        else hipLaunchKernelGGL(place_copy_kernel<float>, dim3(g), dim3(256), 0, st, src, n, (float*)dst);
    }
    SPT_LAUNCH_CHECK();
}

template <int XM>
static void gemv_launch(const PkGemvArgs& a, hipStream_t s) {
    if (a.Npad % 256 || a.K % a.ksplit) throw std::runtime_error("pk_gemv: bad shape");
    const int KC = a.K / a.ksplit;
    dim3 grid(a.Npad / 256, a.ksplit);
#define PK_GEMV_BM(BMV)                                                                                   \
    if (a.B <= BMV) {                                                                                     \
        hipLaunchKernelGGL((gemv_t_kernel<XM, BMV>), grid, dim3(256), (size_t)KC * BMV * 4, s, a);        \
        SPT_LAUNCH_CHECK();                                                                               \
        return;                                                                                           \
    }
    PK_GEMV_BM(4) PK_GEMV_BM(8) PK_GEMV_BM(16) PK_GEMV_BM(32) PK_GEMV_BM(64)
#undef PK_GEMV_BM
    throw std::runtime_error("pk_gemv: more than 64 rows");
}

void pk_gemv(int xmode, const PkGemvArgs& a, hipStream_t s) {
    switch (xmode) {
        case PKX_LSTM0: gemv_launch<PKX_LSTM0>(a, s); return;
        case PKX_LSTM1: gemv_launch<PKX_LSTM1>(a, s); return;
        case PKX_PRED: gemv_launch<PKX_PRED>(a, s); return;
        case PKX_JOINT: gemv_launch<PKX_JOINT>(a, s); return;
    }
    throw std::runtime_error("pk_gemv: bad mode");
}

void pk_lstm_cell(const float* part, int ksplit, int Npad, const float* b_ih, const float* b_hh, int B, int P,
                  const PkState* st, float* h, float* c, hipStream_t s) {
    hipLaunchKernelGGL(lstm_cell_kernel, dim3(cdiv(B * P, 256)), dim3(256), 0, s, part, ksplit, Npad, b_ih, b_hh, B, P,
                       st, h, c);
    SPT_LAUNCH_CHECK();
}

void pk_joint_fin(const PkFinArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(joint_fin_kernel, dim3(a.B), dim3(256), 0, s, a);
    SPT_LAUNCH_CHECK();
}

void pk_state_init(PkState* st, int B, int V, float* h, float* c, int n, hipStream_t s) {
    hipLaunchKernelGGL(state_init_kernel, dim3(cdiv(std::max(B, n), 256)), dim3(256), 0, s, st, B, V, h, c, n);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
