/*
 * wo_mel.c -- TEST INFRASTRUCTURE (oracle). CPU restatement of whisper.cpp's
 * log-mel front end (upstream whisper.cpp ~v1.7.x, vendored by whisper-rs-sys
 * 0.11.1, /root/reference/src-tauri/Cargo.lock:8165-8174; not present in
 * /root/reference).  Compiled with -ffp-contract=off so every float expression
 * rounds exactly as written (the HIP mel kernel mirrors the same expression
 * order with contraction off; tests check it bit-for-bit).
 *
 * Restated pieces:
 *   whisper_global_cache::fill_sin_cos_table / fill_hann_window   -> wo_tables
 *   dft() / fft() (radix-2 DIT, odd N -> naive DFT from the tables) -> fft_rec
 *   log_mel_spectrogram_worker_thread (hann * x, |X|^2, mel dot in
 *     float groups of 4 summed into a double, log10(max(sum,1e-10)))
 *   log_mel_spectrogram (200-sample reflective head, 30 s zero tail,
 *     n_len = (n + 480000)/160 frames, frames past (n+200)/160+1 = -10,
 *     global max - 8 clamp, (x + 4)/4) over the WHOLE input     -> wo_mel_full
 *     (whisper_pcm_to_mel runs once per whisper_full call; each window's
 *     encoder takes frames [seek, seek + 3000)); its first window  -> wo_mel
 * The reference app feeds this 16 kHz mono f32 (src-tauri/src/managers/audio.rs:466-475
 * pads clips < 1 s to 20 000 samples; src-tauri/src/managers/transcription.rs:412-416
 * returns "" for empty audio without calling the engine).
 *
 * WO_MEL_HF restates HF transformers' WhisperFeatureExtractor._np_extract_fbank_features
 * (center=True reflect padding on both ends, 3001 frames with the last dropped,
 * max over the 3000 kept frames) -- used only to pin this file against HF fixtures.
 */
#include "whisper_oracle.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>

#define N_FFT 400
#define HOP 160
#define N_BINS 201
#define SR 16000
#define CHUNK 480000
#define N_FRAMES 3000

static float g_sin[N_FFT], g_cos[N_FFT], g_hann[N_FFT];
static int g_init = 0;

static void init_tables(void) {
    if (g_init) return;
    for (int i = 0; i < N_FFT; i++) {
        double theta = (2 * M_PI * i) / N_FFT;
        g_sin[i] = sinf((float)theta);
        g_cos[i] = cosf((float)theta);
    }
    for (int i = 0; i < N_FFT; i++) {
        /* periodic Hann: offset 0 */
        g_hann[i] = (float)(0.5 * (1.0 - cosf((float)((2.0 * M_PI * i) / (N_FFT)))));
    }
    g_init = 1;
}

void wo_tables(float* hann, float* sin_vals, float* cos_vals) {
    init_tables();
    if (hann) memcpy(hann, g_hann, sizeof g_hann);
    if (sin_vals) memcpy(sin_vals, g_sin, sizeof g_sin);
    if (cos_vals) memcpy(cos_vals, g_cos, sizeof g_cos);
}

/* slaney mel scale (librosa / HF audio_utils.hertz_to_mel, mel_scale="slaney") */
static double hz_to_mel(double f) {
    const double min_log_hz = 1000.0, min_log_mel = 15.0, logstep = 27.0 / log(6.4);
    double m = 3.0 * f / 200.0;
    if (f >= min_log_hz) m = min_log_mel + log(f / min_log_hz) * logstep;
    return m;
}
static double mel_to_hz(double m) {
    const double min_log_hz = 1000.0, min_log_mel = 15.0, logstep = log(6.4) / 27.0;
    double f = 200.0 * m / 3.0;
    if (m >= min_log_mel) f = min_log_hz * exp(logstep * (m - min_log_mel));
    return f;
}

/* mel filters [n_mels][201] float, slaney-normalised triangles over 0..8 kHz */
void wo_mel_filters(int n_mels, float* out) {
    double mel_min = hz_to_mel(0.0), mel_max = hz_to_mel(8000.0);
    double* ff = (double*)malloc(sizeof(double) * (n_mels + 2));
    for (int i = 0; i < n_mels + 2; i++) {
        double mm = mel_min + (mel_max - mel_min) * i / (double)(n_mels + 1);
        if (i == n_mels + 1) mm = mel_max;
        ff[i] = mel_to_hz(mm);
    }
    for (int j = 0; j < n_mels; j++) {
        double enorm = 2.0 / (ff[j + 2] - ff[j]);
        for (int k = 0; k < N_BINS; k++) {
            double fk = (double)(SR / 2) * k / (double)(N_BINS - 1);
            double down = -(ff[j] - fk) / (ff[j + 1] - ff[j]);
            double up = (ff[j + 2] - fk) / (ff[j + 2] - ff[j + 1]);
            double v = down < up ? down : up;
            if (v < 0) v = 0;
            out[j * N_BINS + k] = (float)(v * enorm);
        }
    }
    free(ff);
}

/* whisper.cpp dft(): naive DFT of a real sequence from the 400-entry tables */
static void dft(const float* in, int N, float* out) {
    const int step = N_FFT / N;
    for (int k = 0; k < N; k++) {
        float re = 0, im = 0;
        for (int n = 0; n < N; n++) {
            int idx = (k * n * step) % N_FFT;
            re += in[n] * g_cos[idx];
            im -= in[n] * g_sin[idx];
        }
        out[k * 2 + 0] = re;
        out[k * 2 + 1] = im;
    }
}

/* whisper.cpp fft(): in has room for 2N floats, out for 8N (scratch layout as upstream) */
static void fft_rec(float* in, int N, float* out) {
    if (N == 1) { out[0] = in[0]; out[1] = 0; return; }
    const int half = N / 2;
    if (N - half * 2 == 1) { dft(in, N, out); return; }
    float* even = in + N;
    for (int i = 0; i < half; ++i) even[i] = in[2 * i];
    float* even_fft = out + 2 * N;
    fft_rec(even, half, even_fft);
    float* odd = even;
    for (int i = 0; i < half; ++i) odd[i] = in[2 * i + 1];
    float* odd_fft = even_fft + N;
    fft_rec(odd, half, odd_fft);
    const int step = N_FFT / N;
    for (int k = 0; k < half; k++) {
        int idx = k * step;
        float re = g_cos[idx];
        float im = -g_sin[idx];
        float re_odd = odd_fft[2 * k + 0];
        float im_odd = odd_fft[2 * k + 1];
        out[2 * k + 0] = even_fft[2 * k + 0] + re * re_odd - im * im_odd;
        out[2 * k + 1] = even_fft[2 * k + 1] + re * im_odd + im * re_odd;
        out[2 * (k + half) + 0] = even_fft[2 * k + 0] - re * re_odd + im * im_odd;
        out[2 * (k + half) + 1] = even_fft[2 * k + 1] - re * im_odd - im * re_odd;
    }
}

/* one frame: windowed samples -> log10 mel column (whisper.cpp worker body) */
static void mel_frame(const float* filt, int n_mels, const float* frame, int n_valid,
                      float* fin, float* fout, float* col) {
    for (int j = 0; j < N_FFT; j++) fin[j] = j < n_valid ? g_hann[j] * frame[j] : 0.0f;
    for (int j = N_FFT; j < 2 * N_FFT; j++) fin[j] = 0.0f;
    fft_rec(fin, N_FFT, fout);
    for (int j = 0; j < N_BINS; j++)
        fout[j] = (fout[2 * j + 0] * fout[2 * j + 0] + fout[2 * j + 1] * fout[2 * j + 1]);
    for (int j = 0; j < n_mels; j++) {
        double sum = 0.0;
        int k = 0;
        const float* fr = filt + j * N_BINS;
        for (k = 0; k < N_BINS - 3; k += 4)
            sum += fout[k + 0] * fr[k + 0] + fout[k + 1] * fr[k + 1] +
                   fout[k + 2] * fr[k + 2] + fout[k + 3] * fr[k + 3];
        for (; k < N_BINS; k++) sum += fout[k] * fr[k];
        sum = log10(sum > 1e-10 ? sum : 1e-10);
        col[j] = (float)sum;
    }
}

int wo_mel_len(int n_samples) { return (int)(((long)n_samples + CHUNK) / HOP); }

/* log_mel_spectrogram over the whole input: [n_mels][n_len] normalised (global max - 8) */
static int mel_whole(int n_mels, const float* filt, const float* pcm, int n_samples, float* mel) {
    /* samples_padded = [reflect 200][x][zeros 480000 + 200] */
    const long n_pad = (long)n_samples + CHUNK + 2 * (N_FFT / 2);
    float* sp = (float*)calloc(n_pad, sizeof(float));
    if (!sp) return -3;
    memcpy(sp + N_FFT / 2, pcm, sizeof(float) * n_samples);
    for (int i = 0; i < N_FFT / 2; i++) {
        int src = N_FFT / 2 - i; /* reverse_copy(samples+1, samples+1+200) */
        sp[i] = src < n_samples ? pcm[src] : 0.0f;
    }
    const int n_len = (int)((n_pad - N_FFT) / HOP);
    const int n_sig = n_samples + N_FFT / 2;
    int n_comp = n_sig / HOP + 1;
    if (n_comp > n_len) n_comp = n_len;
    #pragma omp parallel
    {
        float fin[2 * N_FFT], fout[8 * N_FFT], col[256];
        #pragma omp for schedule(static)
        for (int i = 0; i < n_len; i++) {
            if (i < n_comp) {
                const long off = (long)i * HOP;
                int nv = (int)(n_sig - off);
                if (nv > N_FFT) nv = N_FFT;
                mel_frame(filt, n_mels, sp + off, nv, fin, fout, col);
                for (int j = 0; j < n_mels; j++) mel[(size_t)j * n_len + i] = col[j];
            } else {
                for (int j = 0; j < n_mels; j++) mel[(size_t)j * n_len + i] = (float)log10(1e-10);
            }
        }
    }
    double mmax = -1e20;
    for (size_t i = 0; i < (size_t)n_mels * n_len; i++)
        if (mel[i] > mmax) mmax = mel[i];
    mmax -= 8.0;
    for (size_t i = 0; i < (size_t)n_mels * n_len; i++) {
        float v = mel[i];
        if (v < mmax) v = (float)mmax;
        mel[i] = (float)((v + 4.0) / 4.0);
    }
    free(sp);
    return 0;
}

int wo_mel_full(int n_mels, const float* pcm, int n_samples, float* out) {
    if (n_samples < 0) return -1;
    init_tables();
    float* filt = (float*)malloc(sizeof(float) * n_mels * N_BINS);
    wo_mel_filters(n_mels, filt);
    const int rc = mel_whole(n_mels, filt, pcm, n_samples, out);
    free(filt);
    return rc;
}

int wo_mel(int n_mels, const float* pcm, int n_samples, int mode, float* out) {
    if (n_samples < 0 || n_samples > CHUNK) return -1;
    init_tables();
    float* filt = (float*)malloc(sizeof(float) * n_mels * N_BINS);
    wo_mel_filters(n_mels, filt);
    int rc = 0;
    if (mode == WO_MEL_WHISPER_CPP) {
        /* the first window of the whole-input log-mel (n_len >= 3000 frames) */
        const int n_len = wo_mel_len(n_samples);
        float* mel = (float*)malloc(sizeof(float) * (size_t)n_mels * n_len);
        rc = mel_whole(n_mels, filt, pcm, n_samples, mel);
        for (int j = 0; rc == 0 && j < n_mels; j++)
            memcpy(out + (size_t)j * N_FRAMES, mel + (size_t)j * n_len, sizeof(float) * N_FRAMES);
        free(mel);
    } else if (mode == WO_MEL_HF) {
        /* HF: pad/truncate to 480000, centre reflect pad 200 both sides, 3000 frames */
        const int n = CHUNK, pad = N_FFT / 2;
        float* sp = (float*)calloc(n + 2 * pad, sizeof(float));
        for (int i = 0; i < n; i++) sp[pad + i] = i < n_samples ? pcm[i] : 0.0f;
        for (int i = 0; i < pad; i++) {
            sp[i] = sp[2 * pad - i];                     /* x[pad - i]     */
            sp[pad + n + i] = sp[pad + n - 2 - i];       /* x[n - 2 - i]   */
        }
        float* mel = (float*)malloc(sizeof(float) * n_mels * N_FRAMES);
        #pragma omp parallel
        {
            float fin[2 * N_FFT], fout[8 * N_FFT], col[256];
            #pragma omp for schedule(static)
            for (int i = 0; i < N_FRAMES; i++) {
                mel_frame(filt, n_mels, sp + i * HOP, N_FFT, fin, fout, col);
                for (int j = 0; j < n_mels; j++) mel[j * N_FRAMES + i] = col[j];
            }
        }
        double mmax = -1e20;
        for (int i = 0; i < n_mels * N_FRAMES; i++)
            if (mel[i] > mmax) mmax = mel[i];
        mmax -= 8.0;
        for (int i = 0; i < n_mels * N_FRAMES; i++) {
            float v = mel[i];
            if (v < mmax) v = (float)mmax;
            out[i] = (float)((v + 4.0) / 4.0);
        }
        free(mel);
        free(sp);
    } else {
        rc = -2;
    }
    free(filt);
    return rc;
}
