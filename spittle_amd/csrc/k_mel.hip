// k_mel.hip -- log-mel front end on the GPU.
//
// Replaces whisper.cpp's log_mel_spectrogram / log_mel_spectrogram_worker_thread,
// which run on CPU threads inside whisper_full even when a GPU backend is used
// (called from WhisperEngine::transcribe_samples,
// /root/reference/src-tauri/src/managers/transcription.rs:501-503).
//
// One workgroup = 8 consecutive frames of one chunk.  The 400-point FFT follows
// the upstream decomposition exactly (radix-2 decimation in time down to sixteen
// 25-point DFTs from the 400-entry sin/cos tables, same operand order, FP
// contraction off), the power spectrum and the mel dot product keep upstream's
// float groups of four summed into a double, and log10 runs in double -- so the
// output matches the CPU restatement (oracle/wo_mel.c) bit-for-bit up to libm's
// last-ulp differences in log10.  The mel filterbank is walked only over its
// nonzero groups of four (a zero group adds exactly +0.0 to the double sum).
// A per-utterance maximum is reduced with one atomicMax per workgroup on an
// order-preserving integer key; mel_norm then clamps at max - 8, applies
// (x + 4) / 4 and writes the zero-padded, time-major conv1 input of each
// encoder window: frames [seek, seek + 3000) of its utterance.
//
// The log-mel is computed once over each WHOLE utterance, as whisper.cpp's
// whisper_pcm_to_mel does before whisper_full's seek loop: the reflective head
// is the utterance's own first samples, frames run to (n + 480000) / 160, and
// the clamp uses the utterance's global maximum.  Each window then takes its
// slice (whisper_encode_internal's mel_offset = seek).
#include "common.h"
#include "kernels.h"

#pragma clang fp contract(off)

namespace spt {

namespace {

constexpr int FB = 8;  // frames per workgroup
constexpr int NFFT = 400, HOP = 160, NB = 201;

__device__ __forceinline__ unsigned fkey(float f) {
    unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
    unsigned u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return __uint_as_float(u);
}
__device__ __forceinline__ int frames_computed(int n) {
    const int n_sig = n + NFFT / 2;
    const int n_len = (n + 480000) / HOP;
    return min(n_sig / HOP + 1, n_len);
}

// combine stage of upstream fft(): E = even-half spectrum, O = odd-half spectrum
__device__ __forceinline__ void butterfly(const float* E, const float* O, float* out, int k, int half, float re,
                                          float im, bool upper) {
    const float re_odd = O[2 * k + 0];
    const float im_odd = O[2 * k + 1];
    out[2 * k + 0] = E[2 * k + 0] + re * re_odd - im * im_odd;
    out[2 * k + 1] = E[2 * k + 1] + re * im_odd + im * re_odd;
    if (upper) {
        out[2 * (k + half) + 0] = E[2 * k + 0] - re * re_odd + im * im_odd;
        out[2 * (k + half) + 1] = E[2 * k + 1] - re * im_odd - im * re_odd;
    }
}

__global__ __launch_bounds__(256) void mel_frames_kernel(const float* __restrict__ pcm, MelUtts ut, int n_mels,
                                                         MelTables tb, float* __restrict__ mel_raw,
                                                         unsigned* __restrict__ mel_max) {
    __shared__ float s_smp[FB * HOP + NFFT - HOP];
    __shared__ float s_tab[3][NFFT];
    __shared__ float s_buf[2][FB][2 * NFFT];
    __shared__ unsigned s_max;
    const int b = blockIdx.y, tid = threadIdx.x;
    const int n = ut.n[b];
    const int n_comp = frames_computed(n);
    const int f0 = blockIdx.x * FB;
    if (f0 >= n_comp) return;
    const int nf = min(FB, n_comp - f0);
    const int n_sig = n + NFFT / 2;
    const float* x = pcm + ut.pcm_off[b];
    if (tid == 0) s_max = 0u;
    for (int i = tid; i < NFFT; i += 256) {
        s_tab[0][i] = tb.hann[i];
        s_tab[1][i] = tb.sinv[i];
        s_tab[2][i] = tb.cosv[i];
    }
    // samples_padded = [x[200], x[199], ..., x[1]] [x] [zeros]; positions >= n + 200 are zero
    for (int i = tid; i < FB * HOP + NFFT - HOP; i += 256) {
        const int p = f0 * HOP + i;
        float v = 0.0f;
        if (p < n_sig) {
            if (p < NFFT / 2) {
                const int src = NFFT / 2 - p;
                v = src < n ? x[src] : 0.0f;
            } else {
                v = x[p - NFFT / 2];
            }
        }
        s_smp[i] = v;
    }
    __syncthreads();
    // windowed real input -> s_buf[1][f][0..399]
    for (int i = tid; i < nf * NFFT; i += 256) {
        const int f = i / NFFT, j = i - f * NFFT;
        s_buf[1][f][j] = s_tab[0][j] * s_smp[f * HOP + j];
    }
    __syncthreads();
    // sixteen 25-point DFTs per frame (leaf o holds inputs o + 16 n) -> s_buf[0][f][(o*25 + k)*2]
    for (int i = tid; i < nf * NFFT; i += 256) {
        const int f = i / NFFT, rem = i - f * NFFT;
        const int o = rem / 25, k = rem - o * 25;
        const float* in = &s_buf[1][f][0];
        float re = 0.0f, im = 0.0f;
        for (int nn = 0; nn < 25; nn++) {
            const int idx = (k * nn * 16) % NFFT;
            const float v = in[o + 16 * nn];
            re += v * s_tab[2][idx];
            im -= v * s_tab[1][idx];
        }
        s_buf[0][f][(o * 25 + k) * 2 + 0] = re;
        s_buf[0][f][(o * 25 + k) * 2 + 1] = im;
    }
    __syncthreads();
    // radix-2 levels: size N subproblem at offset o combines (o) and (o + 400/N) of size N/2
    int src = 0;
#pragma unroll 1
    for (int N = 50; N <= NFFT; N *= 2) {
        const int half = N / 2, nsub = NFFT / N, tw = NFFT / N;
        const bool last = (N == NFFT);
        for (int i = tid; i < nf * nsub * half; i += 256) {
            const int f = i / (nsub * half), rem = i - f * nsub * half;
            const int o = rem / half, k = rem - o * half;
            const float* E = &s_buf[src][f][2 * (o * half)];
            const float* O = &s_buf[src][f][2 * ((o + nsub) * half)];
            float* out = &s_buf[src ^ 1][f][2 * (o * N)];
            const float re = s_tab[2][k * tw];
            const float im = -s_tab[1][k * tw];
            butterfly(E, O, out, k, half, re, im, !last || k == 0);
        }
        src ^= 1;
        __syncthreads();
    }
    // power spectrum (bins 0..200) in place
    for (int i = tid; i < nf * NB; i += 256) {
        const int f = i / NB, j = i - f * NB;
        const float re = s_buf[src][f][2 * j + 0], im = s_buf[src][f][2 * j + 1];
        s_buf[src ^ 1][f][j] = re * re + im * im;
    }
    __syncthreads();
    float lmax = -INFINITY;
    for (int i = tid; i < nf * n_mels; i += 256) {
        const int f = i / n_mels, j = i - f * n_mels;
        const float* pw = &s_buf[src ^ 1][f][0];
        const float* fl = tb.filt + (size_t)j * NB;
        const int g0 = tb.grp[2 * j], g1 = tb.grp[2 * j + 1];
        double sum = 0.0;
        for (int gi = g0; gi < g1; gi++) {
            if (gi < 50) {
                const int k = 4 * gi;
                sum += pw[k + 0] * fl[k + 0] + pw[k + 1] * fl[k + 1] + pw[k + 2] * fl[k + 2] + pw[k + 3] * fl[k + 3];
            } else {
                sum += pw[200] * fl[200];
            }
        }
        const float v = (float)log10(sum > 1e-10 ? sum : 1e-10);
        mel_raw[(size_t)(ut.row_off[b] + f0 + f) * n_mels + j] = v;
        lmax = fmaxf(lmax, v);
    }
    lmax = wave_max(lmax);
    if ((tid & 63) == 0) atomicMax(&s_max, fkey(lmax));
    __syncthreads();
    if (tid == 0) atomicMax(&mel_max[b], s_max);
}

template <typename T>
__global__ void mel_norm_kernel(const float* __restrict__ mel_raw, const unsigned* __restrict__ mel_max, MelUtts ut,
                                const int* __restrict__ win_utt, const int* __restrict__ win_seek, int n_mels, int Cp,
                                T* __restrict__ out, float* __restrict__ dbg) {
    const int b = blockIdx.y;  // encoder row (window)
    const int r = blockIdx.x;  // padded row 0..3001
    const int u = win_utt[b], seek = win_seek[b];
    const int n_comp = frames_computed(ut.n[u]);
    float gmax = fkey_inv(mel_max[u]);
    if (!(gmax > -10.0f)) gmax = -10.0f;  // frames past the signal are log10(1e-10)
    const double mmax = (double)gmax - 8.0;
    const int t = r - 1, f = seek + t;  // f < n_len = n / 160 + 3000 whenever seek < n_len_org
    for (int c = threadIdx.x; c < Cp; c += blockDim.x) {
        float o = 0.0f;
        if (t >= 0 && t < 3000 && c < n_mels) {
            float v = f < n_comp ? mel_raw[(size_t)(ut.row_off[u] + f) * n_mels + c] : -10.0f;
            if ((double)v < mmax) v = (float)mmax;
            o = (float)(((double)v + 4.0) / 4.0);
            if (dbg) dbg[((size_t)b * n_mels + c) * 3000 + t] = o;
        }
        out[((size_t)b * MEL_ROWS + r) * Cp + c] = from_f<T>(o);
    }
}

}  // namespace

int mel_rows(int n) {
    const int n_sig = n + NFFT / 2, n_len = (int)(((int64_t)n + 480000) / HOP);
    return std::min(n_sig / HOP + 1, n_len);
}

void mel_frames(const float* pcm, MelUtts u, int U, int max_rows, int n_mels, MelTables t, float* mel_raw,
                unsigned* mel_max, hipStream_t st) {
    HIP_CHECK(hipMemsetAsync(mel_max, 0, sizeof(unsigned) * U, st));
    if (U < 1 || max_rows < 1) return;
    dim3 grid(cdiv(max_rows, FB), U);
    hipLaunchKernelGGL(mel_frames_kernel, grid, dim3(256), 0, st, pcm, u, n_mels, t, mel_raw, mel_max);
    SPT_LAUNCH_CHECK();
}

void mel_norm(int dtype, const float* mel_raw, const unsigned* mel_max, MelUtts u, const int* win_utt,
              const int* win_seek, int E, int n_mels, int Cp, void* mel_in, float* dbg, hipStream_t st) {
    dim3 grid(MEL_ROWS, E);
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(mel_norm_kernel<bf16>, grid, dim3(128), 0, st, mel_raw, mel_max, u, win_utt, win_seek,
                           n_mels, Cp, (bf16*)mel_in, dbg);
    else
        hipLaunchKernelGGL(mel_norm_kernel<float>, grid, dim3(128), 0, st, mel_raw, mel_max, u, win_utt, win_seek,
                           n_mels, Cp, (float*)mel_in, dbg);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
