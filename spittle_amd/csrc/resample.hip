// resample.hip -- capture-side resampler: the spt_resampler_* half of
// include/spittle_hip.h (ABI 7).
//
// Replaces Spittle's FrameResampler (/root/reference/src-tauri/src/audio_toolkit/audio/
// resampler.rs:7-104) over rubato 0.16.2 FftFixedIn<f32>(in_hz, out_hz, 1024, 1, 1), fed by the
// recorder (recorder.rs:264-268 new, :330 push, :355 finish).  rubato's unit is linear in its
// fft_size_in input samples: zero-pad to 2 * nin, real FFT, multiply by the filter spectrum,
// keep bins [0, new_len), unnormalised inverse real FFT of 2 * nout samples; the first nout plus
// the previous unit's last nout are the output.  So the whole unit is one real matrix
// M [nin][2 nout] = F diag(H) G, built once per context on the device in f64, and a stream of
// U units is one f32 GEMM [U][nin] x M (exact-f32 MFMA, gemm_nt) followed by an overlap-add:
//   units_kernel   input -> [U][Kp] unit rows (K padded to the GEMM's 32-element alignment)
//   gemm_nt        [U][Kp] x W[Np][Kp]^T -> Y [U][Np]   (W = M^T, zero rows/columns as padding)
//   ola_kernel     out[u nout + m] = Y[u][m] + Y[u-1][nout + m], zero-padded to whole frames
// Filter and sizes follow oracle/resampler.py (the CPU restatement this path is tested against).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <memory>
#include <new>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/spittle_hip.h"
#include "common.h"
#include "kernels.h"

namespace spt {
namespace {

// M^T [Np][Kp] (f32): row m (output sample of a unit), column j (input sample of a unit) is
// y_m for a unit impulse at j:  y_m = sum_k c_k Re(H_k e^{-2 pi i j k / (2 nin)} e^{2 pi i k m / (2 nout)})
// over the kept bins k < new_len (c_0 = 1, c_k = 2 below the output Nyquist bin, which is 1).
// Angles are reduced exactly in integers before sincospi (f64).
__global__ __launch_bounds__(256) void rs_matrix_kernel(const double2* __restrict__ hf, int nin, int nout,
                                                         int new_len, int Kp, float* __restrict__ wt) {
    const int m = blockIdx.y;
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= Kp) return;
    double acc = 0.0;
    if (j < nin && m < 2 * nout) {
        const long n2i = 2L * nin, n2o = 2L * nout;
        for (int k = 0; k < new_len; ++k) {
            // phase / pi = 2 (k m / n2o - j k / n2i) = 2 (k m n2i - j k n2o) / (n2i n2o), reduced mod 2
            const long p = ((long)k * m % n2o) * n2i - ((long)j * k % n2i) * n2o;
            const long den = n2i * n2o;
            long r = p % den;
            if (r < 0) r += den;
            double s, c;
            sincospi(2.0 * (double)r / (double)den, &s, &c);
            const double2 h = hf[k];
            const double re = h.x * c - h.y * s;  // Re(H e^{i phase})
            const double w = (k == 0 || k == nout) ? 1.0 : 2.0;
            acc += w * re;
        }
    }
    wt[(size_t)m * Kp + j] = (float)acc;
}

__global__ __launch_bounds__(256) void units_kernel(const float* __restrict__ x, int64_t n, int nin, int Kp,
                                                    float* __restrict__ a) {
    const int u = blockIdx.x;
    float* row = a + (size_t)u * Kp;
    for (int j = threadIdx.x; j < Kp; j += 256) {
        const int64_t s = (int64_t)u * nin + j;
        row[j] = (j < nin && s < n) ? x[s] : 0.0f;
    }
}

__global__ __launch_bounds__(256) void ola_kernel(const float* __restrict__ y, int U, int nout, int Np, int64_t n_out,
                                                  float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_out) return;
    const int64_t u = i / nout;
    const int m = (int)(i - u * nout);
    float v = 0.0f;
    if (u < U) {
        v = y[(size_t)u * Np + m];
        if (u > 0) v += y[(size_t)(u - 1) * Np + nout + m];
    }
    out[i] = v;
}

__global__ __launch_bounds__(256) void copy_pad_kernel(const float* __restrict__ x, int64_t n, int64_t n_out,
                                                       float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n_out) out[i] = i < n ? x[i] : 0.0f;
}

int64_t roundup(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace
}  // namespace spt

struct spt_resampler {
    int in_hz = 0, out_hz = 0, frame_samples = 0, chunk_in = 1024, device = 0;
    int nin = 0, nout = 0, new_len = 0, Kp = 0, Np = 0;
    float* wt = nullptr;        // M^T [Np][Kp]
    float* work = nullptr;      // x | units | Y | out, sized for `cap_units`
    int64_t cap_units = -1;
    hipStream_t st = nullptr;
    std::string err;
    ~spt_resampler() {
        (void)hipSetDevice(device);
        if (wt) (void)hipFree(wt);
        if (work) (void)hipFree(work);
        if (st) (void)hipStreamDestroy(st);
    }
};

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
    if (err && errlen) {
        strncpy(err, m.c_str(), errlen - 1);
        err[errlen - 1] = 0;
    }
}

// rubato FftFixedIn filter (oracle/resampler.py filter_taps): Blackman-Harris^2-windowed sinc,
// fft_size_in taps centred at nin / 2, unit sum, divided by 2 nin; its spectrum over 2 nin points
std::vector<double> filter_spectrum(int nin, int nout) {
    const double PI = 3.14159265358979323846;
    double fc = pow(0.4, 16.0 / nin);
    if (nin > nout) fc *= (double)nout / nin;
    std::vector<double> h(nin);
    double sum = 0.0;
    for (int x = 0; x < nin; ++x) {
        const double t = (double)x / nin;
        double w = 0.35875 - 0.48829 * cos(2 * PI * t) + 0.14128 * cos(4 * PI * t) - 0.01168 * cos(6 * PI * t);
        w *= w;
        const double a = (x - nin / 2) * fc;
        const double s = a == 0.0 ? 1.0 : sin(PI * a) / (PI * a);
        h[x] = w * s;
        sum += h[x];
    }
    for (double& v : h) v /= sum * 2.0 * nin;
    std::vector<double> hf(2 * (size_t)(nin + 1));
    for (int k = 0; k <= nin; ++k) {  // H_k = sum_x h_x e^{-2 pi i x k / (2 nin)}
        double re = 0.0, im = 0.0;
        for (int x = 0; x < nin; ++x) {
            const long r = ((long)x * k) % (2L * nin);
            const double ang = PI * (double)r / nin;
            re += h[x] * cos(ang);
            im -= h[x] * sin(ang);
        }
        hf[2 * k] = re;
        hf[2 * k + 1] = im;
    }
    return hf;
}

}  // namespace

extern "C" {

spt_status spt_resampler_create(int32_t in_hz, int32_t out_hz, int32_t frame_samples, int32_t device,
                                spt_resampler** out, char* err, size_t errlen) {
    if (!out) {
        set_err(err, errlen, "null argument");
        return SPT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    if (in_hz < 1000 || in_hz > 384000 || out_hz < 1000 || out_hz > 384000) {
        set_err(err, errlen, "sample rates must be in [1000, 384000] Hz");
        return SPT_ERR_INVALID_ARG;
    }
    if (frame_samples < 1 || frame_samples > (1 << 20)) {
        set_err(err, errlen, "frame_samples must be in [1, 2^20] (FrameResampler: frame duration too short)");
        return SPT_ERR_INVALID_ARG;
    }
    std::unique_ptr<spt_resampler> r(new (std::nothrow) spt_resampler());
    if (!r) return SPT_ERR_OOM;
    r->in_hz = in_hz;
    r->out_hz = out_hz;
    r->frame_samples = frame_samples;
    r->device = device;
    try {
        HIP_CHECK(hipSetDevice(device));
        HIP_CHECK(hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking));
        if (in_hz != out_hz) {
            const int g = std::gcd(in_hz, out_hz);
            const int fft_chunks = (r->chunk_in + in_hz / g - 1) / (in_hz / g);
            r->nin = fft_chunks * (in_hz / g);
            r->nout = fft_chunks * (out_hz / g);
            if (r->nin > 16384 || r->nout > 16384) {
                set_err(err, errlen, "resampling ratio needs an FFT unit above 16384 samples");
                return SPT_ERR_UNSUPPORTED;
            }
            r->new_len = r->nin > r->nout ? r->nout : r->nin + 1;
            r->Kp = (int)spt::roundup(r->nin, 32);
            r->Np = (int)spt::roundup(2 * r->nout, 128);
            const std::vector<double> hf = filter_spectrum(r->nin, r->nout);
            double2* d_hf = nullptr;
            HIP_CHECK(hipMalloc(&d_hf, hf.size() * sizeof(double)));
            HIP_CHECK(hipMemcpy(d_hf, hf.data(), hf.size() * sizeof(double), hipMemcpyHostToDevice));
            HIP_CHECK(hipMalloc(&r->wt, (size_t)r->Np * r->Kp * 4));
            hipLaunchKernelGGL(spt::rs_matrix_kernel, dim3(spt::cdiv(r->Kp, 256), r->Np), dim3(256), 0, r->st, d_hf,
                               r->nin, r->nout, r->new_len, r->Kp, r->wt);
            SPT_LAUNCH_CHECK();
            HIP_CHECK(hipStreamSynchronize(r->st));
            HIP_CHECK(hipFree(d_hf));
        }
    } catch (const std::exception& e) {
        set_err(err, errlen, e.what());
        return dynamic_cast<const std::bad_alloc*>(&e) ? SPT_ERR_OOM : SPT_ERR_DEVICE;
    }
    *out = r.release();
    return SPT_OK;
}

spt_status spt_resampler_info(const spt_resampler* r, int32_t* fft_size_in, int32_t* fft_size_out) {
    if (!r) return SPT_ERR_INVALID_ARG;
    if (fft_size_in) *fft_size_in = r->nin;
    if (fft_size_out) *fft_size_out = r->nout;
    return SPT_OK;
}

size_t spt_resample_output_len(const spt_resampler* r, size_t n_samples) {
    if (!r || n_samples == 0) return 0;
    const int64_t fs = r->frame_samples;
    int64_t produced = (int64_t)n_samples;
    if (r->in_hz != r->out_hz) {
        const int64_t n_proc = spt::roundup((int64_t)n_samples, r->chunk_in);  // finish pads the last chunk
        produced = n_proc / r->nin * r->nout;
    }
    return (size_t)spt::roundup(produced, fs);  // finish pads the pending frame
}

spt_status spt_resample(spt_resampler* r, const float* pcm, size_t n_samples, float* out, size_t out_cap,
                        size_t* n_out) {
    if (!r || (!pcm && n_samples) || !n_out) return SPT_ERR_INVALID_ARG;
    const size_t need = spt_resample_output_len(r, n_samples);
    *n_out = need;
    if (need == 0) return SPT_OK;
    if (!out || out_cap < need) {
        r->err = "output buffer too small: need " + std::to_string(need) + " samples";
        return SPT_ERR_INVALID_ARG;
    }
    try {
        HIP_CHECK(hipSetDevice(r->device));
        const int64_t n = (int64_t)n_samples;
        const int64_t U = r->in_hz != r->out_hz ? spt::roundup(n, r->chunk_in) / r->nin : 0;
        // workspace: x [n] | units [U][Kp] | Y [U][Np] | out [need]  (f32, 256-B carved)
        auto al = [](int64_t e) { return spt::roundup(e, 64); };
        const int64_t total = al(n) + al(U * r->Kp) + al(U * r->Np) + al((int64_t)need);
        if (total > r->cap_units) {
            if (r->work) HIP_CHECK(hipFree(r->work));
            r->work = nullptr;
            HIP_CHECK(hipMalloc(&r->work, (size_t)total * 4));
            r->cap_units = total;
        }
        float* x = r->work;
        float* a = x + al(n);
        float* y = a + al(U * r->Kp);
        float* o = y + al(U * r->Np);
        HIP_CHECK(hipMemcpyAsync(x, pcm, (size_t)n * 4, hipMemcpyHostToDevice, r->st));
        const int64_t nblk = ((int64_t)need + 255) / 256;
        if (r->in_hz == r->out_hz) {
            hipLaunchKernelGGL(spt::copy_pad_kernel, dim3((unsigned)nblk), dim3(256), 0, r->st, x, n, (int64_t)need, o);
            SPT_LAUNCH_CHECK();
        } else {
            if (U > 0) {
                hipLaunchKernelGGL(spt::units_kernel, dim3((unsigned)U), dim3(256), 0, r->st, x, n, r->nin, r->Kp, a);
                SPT_LAUNCH_CHECK();
                spt::GemmArgs g{};
                g.A = a; g.lda = r->Kp; g.W = r->wt; g.ldw = r->Kp;
                g.M = (int)U; g.N = r->Np; g.K = r->Kp; g.bias = nullptr; g.C = y; g.ldc = r->Np;
                spt::gemm_nt(spt::DT_F32, spt::EPI_BIAS, g, 1, r->st);
            }
            hipLaunchKernelGGL(spt::ola_kernel, dim3((unsigned)nblk), dim3(256), 0, r->st, y, (int)U, r->nout, r->Np,
                               (int64_t)need, o);
            SPT_LAUNCH_CHECK();
        }
        HIP_CHECK(hipMemcpyAsync(out, o, need * 4, hipMemcpyDeviceToHost, r->st));
        HIP_CHECK(hipStreamSynchronize(r->st));
    } catch (const std::exception& e) {
        r->err = e.what();
        return dynamic_cast<const std::bad_alloc*>(&e) ? SPT_ERR_OOM : SPT_ERR_DEVICE;
    }
    return SPT_OK;
}

const char* spt_resampler_last_error(const spt_resampler* r) { return r ? r->err.c_str() : "null resampler"; }

void spt_resampler_destroy(spt_resampler* r) { delete r; }

}  // extern "C"
