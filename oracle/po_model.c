/*
 * po_model.c -- TEST INFRASTRUCTURE (oracle).  fp32 CPU restatement of the Parakeet-V3
 * (FastConformer + TDT) path Spittle runs through transcribe-rs' ParakeetEngine
 * (/root/reference/src-tauri/src/managers/transcription.rs:278-297, 505-513).  The model
 * definition is NeMo's, restated [upstream, recalled]; see parakeet_oracle.h for the list.
 * Every function below names the NeMo module it restates.
 *
 * Synthetic weights: value = u * 2^e (+ 1 for gains), u from the splitmix64 stream shared with
 * wo_model.c and the device generator (spittle_amd/csrc/k_init.hip); matrices of the encoder's
 * linear layers are bf16- or fp16-rounded (RNE) for the bf16 / fp16 engine; convolution taps, norms, biases, the
 * prediction network and the joint stay f32 on both sides.
 */
#include "parakeet_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ PRNG (as wo_model.c) */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline float urand(uint64_t seed, uint32_t tid, uint64_t i) {
    uint64_t x = i + ((uint64_t)tid << 32) + seed * 0xD1B54A32D192ED03ULL;
    return (float)(uint32_t)(mix64(x) >> 40) * (1.0f / 8388608.0f) - 1.0f;
}
static inline float bf16_round(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
    memcpy(&f, &u, 4);
    return f;
}
/* IEEE half round-to-nearest-even, subnormals included (the device's v_cvt_f16_f32) */
static inline float f16_round(float f) {
    if (!isfinite(f) || f == 0.0f) return f;
    const float a = fabsf(f);
    float q;
    if (a < 6.103515625e-05f) q = 5.9604644775390625e-08f;  /* 2^-14 normal floor; 2^-24 quantum */
    else {
        int ex;
        frexpf(a, &ex);          /* a = m 2^ex, m in [0.5, 1): 11 significant bits -> quantum 2^(ex-11) */
        q = ldexpf(1.0f, ex - 11);
    }
    const float r = nearbyintf(a / q) * q;
    return f < 0 ? -r : r;
}
static int fanin_exp(int K) { return (int)floor(log2(sqrt(3.0 / (double)K)) + 0.5); }

void po_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------ weights */
/* kinds: value = u * 2^e, plus one for PLUS1 (norm gains, BatchNorm variance); MATB: a matrix
 * rounded to bf16 in the bf16 model */
enum { P_MATB = 0, P_MAT, P_SCALE, P_PLUS1 };

typedef struct {
    float *ln_ff1_w, *ln_ff1_b, *ff1_w1, *ff1_b1, *ff1_w2, *ff1_b2;
    float *ln_att_w, *ln_att_b, *q_w, *q_b, *k_w, *k_b, *v_w, *v_b, *o_w, *o_b, *pos_w, *pos_u, *pos_v;
    float *ln_conv_w, *ln_conv_b, *pw1_w, *pw1_b, *dw_w, *dw_b, *bn_g, *bn_b, *bn_m, *bn_v, *pw2_w, *pw2_b;
    float *ln_ff2_w, *ln_ff2_b, *ff2_w1, *ff2_b1, *ff2_w2, *ff2_b2;
    float *ln_out_w, *ln_out_b;
} po_layer;

typedef struct { int tid, kind, e; int64_t n; float** slot; } po_t;

struct po_model {
    po_dims dm;
    uint64_t seed;
    int wdtype;
    float *c0_w, *c0_b, *dw1_w, *dw1_b, *pw1_w, *pw1_b, *dw2_w, *dw2_b, *pw2_w, *pw2_b, *sub_w, *sub_b;
    po_layer* L;
    float *emb, *lstm_wih[2], *lstm_whh[2], *lstm_bih[2], *lstm_bhh[2];
    float *j_enc_w, *j_enc_b, *j_pred_w, *j_pred_b, *j_out_w, *j_out_b;
    int n_t;
    po_t* t;
};

static void add(po_model* m, int tid, int kind, int e, int64_t n, float** slot) {
    po_t* x = &m->t[m->n_t++];
    x->tid = tid; x->kind = kind; x->e = e; x->n = n; x->slot = slot;
}

/* frequency bins left after the three stride-2 convolutions of the subsampling */
static int sub_f3(int n_mels) {
    int f = n_mels;
    for (int i = 0; i < 3; i++) f = (f - 1) / 2 + 1;
    return f;
}

/* Tensor ids (contract with spittle_amd/csrc/parakeet.cpp):
 *   subsampling 1..12; layer l: 1000 + 64 l + {0..38}; prediction network + joint 90000 + {0..14} */
static void build_table(po_model* m) {
    const po_dims* D = &m->dm;
    const int d = D->d, C = D->sub_ch, P = D->pred, H = D->n_heads, dk = d / H, K = D->conv_k;
    const int F3 = sub_f3(D->n_mels), V1 = D->n_vocab + 1, NO = V1 + D->n_dur;
    const int64_t dd = (int64_t)d * d;
    m->t = (po_t*)calloc(64 + 40 * D->n_layers, sizeof(po_t));
    add(m, 1, P_MAT, fanin_exp(9), (int64_t)C * 9, &m->c0_w);
    add(m, 2, P_SCALE, -5, C, &m->c0_b);
    add(m, 3, P_MAT, fanin_exp(9), (int64_t)C * 9, &m->dw1_w);
    add(m, 4, P_SCALE, -5, C, &m->dw1_b);
    add(m, 5, P_MATB, fanin_exp(C), (int64_t)C * C, &m->pw1_w);
    add(m, 6, P_SCALE, -5, C, &m->pw1_b);
    add(m, 7, P_MAT, fanin_exp(9), (int64_t)C * 9, &m->dw2_w);
    add(m, 8, P_SCALE, -5, C, &m->dw2_b);
    add(m, 9, P_MATB, fanin_exp(C), (int64_t)C * C, &m->pw2_w);
    add(m, 10, P_SCALE, -5, C, &m->pw2_b);
    add(m, 11, P_MATB, fanin_exp(C * F3), (int64_t)d * C * F3, &m->sub_w);
    add(m, 12, P_SCALE, -5, d, &m->sub_b);
    for (int l = 0; l < D->n_layers; l++) {
        po_layer* y = &m->L[l];
        const int b = 1000 + 64 * l;
        add(m, b + 0, P_PLUS1, -3, d, &y->ln_ff1_w);
        add(m, b + 1, P_SCALE, -4, d, &y->ln_ff1_b);
        add(m, b + 2, P_MATB, fanin_exp(d), (int64_t)D->ff * d, &y->ff1_w1);
        add(m, b + 3, P_SCALE, -5, D->ff, &y->ff1_b1);
        add(m, b + 4, P_MATB, fanin_exp(D->ff), (int64_t)D->ff * d, &y->ff1_w2);
        add(m, b + 5, P_SCALE, -5, d, &y->ff1_b2);
        add(m, b + 6, P_PLUS1, -3, d, &y->ln_att_w);
        add(m, b + 7, P_SCALE, -4, d, &y->ln_att_b);
        add(m, b + 8, P_MATB, fanin_exp(d), dd, &y->q_w);
        add(m, b + 9, P_SCALE, -5, d, &y->q_b);
        add(m, b + 10, P_MATB, fanin_exp(d), dd, &y->k_w);
        add(m, b + 11, P_SCALE, -5, d, &y->k_b);
        add(m, b + 12, P_MATB, fanin_exp(d), dd, &y->v_w);
        add(m, b + 13, P_SCALE, -5, d, &y->v_b);
        add(m, b + 14, P_MATB, fanin_exp(d), dd, &y->o_w);
        add(m, b + 15, P_SCALE, -5, d, &y->o_b);
        add(m, b + 16, P_MATB, fanin_exp(d), dd, &y->pos_w);
        add(m, b + 17, P_SCALE, -4, (int64_t)H * dk, &y->pos_u);
        add(m, b + 18, P_SCALE, -4, (int64_t)H * dk, &y->pos_v);
        add(m, b + 19, P_PLUS1, -3, d, &y->ln_conv_w);
        add(m, b + 20, P_SCALE, -4, d, &y->ln_conv_b);
        add(m, b + 21, P_MATB, fanin_exp(d), 2 * dd, &y->pw1_w);
        add(m, b + 22, P_SCALE, -5, 2 * d, &y->pw1_b);
        add(m, b + 23, P_MAT, fanin_exp(K), (int64_t)d * K, &y->dw_w);
        add(m, b + 24, P_SCALE, -5, d, &y->dw_b);
        add(m, b + 25, P_PLUS1, -3, d, &y->bn_g);
        add(m, b + 26, P_SCALE, -4, d, &y->bn_b);
        add(m, b + 27, P_SCALE, -4, d, &y->bn_m);
        add(m, b + 28, P_PLUS1, -2, d, &y->bn_v);
        add(m, b + 29, P_MATB, fanin_exp(d), dd, &y->pw2_w);
        add(m, b + 30, P_SCALE, -5, d, &y->pw2_b);
        add(m, b + 31, P_PLUS1, -3, d, &y->ln_ff2_w);
        add(m, b + 32, P_SCALE, -4, d, &y->ln_ff2_b);
        add(m, b + 33, P_MATB, fanin_exp(d), (int64_t)D->ff * d, &y->ff2_w1);
        add(m, b + 34, P_SCALE, -5, D->ff, &y->ff2_b1);
        add(m, b + 35, P_MATB, fanin_exp(D->ff), (int64_t)D->ff * d, &y->ff2_w2);
        add(m, b + 36, P_SCALE, -5, d, &y->ff2_b2);
        add(m, b + 37, P_PLUS1, -3, d, &y->ln_out_w);
        add(m, b + 38, P_SCALE, -4, d, &y->ln_out_b);
    }
    add(m, 90000, P_SCALE, -2, (int64_t)V1 * P, &m->emb);
    for (int j = 0; j < 2; j++) {
        add(m, 90001 + 4 * j, P_MAT, fanin_exp(P), (int64_t)4 * P * P, &m->lstm_wih[j]);
        add(m, 90002 + 4 * j, P_MAT, fanin_exp(P), (int64_t)4 * P * P, &m->lstm_whh[j]);
        add(m, 90003 + 4 * j, P_SCALE, -5, 4 * P, &m->lstm_bih[j]);
        add(m, 90004 + 4 * j, P_SCALE, -5, 4 * P, &m->lstm_bhh[j]);
    }
    add(m, 90009, P_MAT, fanin_exp(d), (int64_t)P * d, &m->j_enc_w);
    add(m, 90010, P_SCALE, -5, P, &m->j_enc_b);
    add(m, 90011, P_MAT, fanin_exp(P), (int64_t)P * P, &m->j_pred_w);
    add(m, 90012, P_SCALE, -5, P, &m->j_pred_b);
    add(m, 90013, P_MAT, fanin_exp(P), (int64_t)NO * P, &m->j_out_w);
    add(m, 90014, P_SCALE, -5, NO, &m->j_out_b);
}

static void gen(const po_model* m, const po_t* t) {
    float* dst = *t->slot;
    const float sc = ldexpf(1.0f, t->e);
    const int round = t->kind == P_MATB ? m->wdtype : PO_W_F32;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < t->n; i++) {
        float v = urand(m->seed, (uint32_t)t->tid, (uint64_t)i) * sc;
        if (t->kind == P_PLUS1) v = 1.0f + v;
        if (round == PO_W_BF16) v = bf16_round(v);
        else if (round == PO_W_F16) v = f16_round(v);
        dst[i] = v;
    }
}

po_model* po_create(const po_dims* dims, uint64_t seed, int wdtype) {
    po_model* m = (po_model*)calloc(1, sizeof(po_model));
    m->dm = *dims;
    m->seed = seed;
    m->wdtype = wdtype;
    m->L = (po_layer*)calloc(dims->n_layers > 0 ? dims->n_layers : 1, sizeof(po_layer));
    build_table(m);
    for (int i = 0; i < m->n_t; i++) {
        *m->t[i].slot = (float*)malloc(sizeof(float) * (size_t)m->t[i].n);
        gen(m, &m->t[i]);
    }
    /* the blank row of the prediction network's embedding is zero (blank_as_pad) */
    memset(m->emb + (size_t)dims->n_vocab * dims->pred, 0, sizeof(float) * dims->pred);
    return m;
}

void po_destroy(po_model* m) {
    if (!m) return;
    for (int i = 0; i < m->n_t; i++) free(*m->t[i].slot);
    free(m->t);
    free(m->L);
    free(m);
}

int64_t po_tensor(po_model* m, int tid, const float** data) {
    for (int i = 0; i < m->n_t; i++)
        if (m->t[i].tid == tid) {
            *data = *m->t[i].slot;
            return m->t[i].n;
        }
    return -1;
}

int po_set_tensor(po_model* m, int tid, const float* data, int64_t n) {
    for (int i = 0; i < m->n_t; i++)
        if (m->t[i].tid == tid) {
            if (m->t[i].n != n) return -1;
            memcpy(*m->t[i].slot, data, sizeof(float) * (size_t)n);
            return 0;
        }
    return -1;
}

/* ------------------------------------------------------------------ preprocessor */
/* valid frames: NeMo FilterbankFeatures.get_seq_len = (n + 2*256 - 512) // 160 (HF
 * feature_extraction_parakeet.py:263-265); the STFT's last centred frame is not one of them */
int po_n_frames(int n) { return n > 0 ? n / 160 : 0; }

/* NeMo FilterbankFeatures (normalize="per_feature", log, mag_power 2, preemph 0.97,
 * n_fft 512, win 400 symmetric Hann, hop 160, centre padding, 128 slaney mels 0-8 kHz) */
static void mel_filters(int n_mels, float* fb /* [n_mels][257] */) {
    /* librosa.filters.mel(sr=16000, n_fft=512, n_mels, fmin=0, fmax=8000, htk=False, norm="slaney") */
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
#define HZ2MEL(f) ((f) < min_log_hz ? (f) / f_sp : min_log_mel + log((f) / min_log_hz) / logstep)
#define MEL2HZ(z) ((z) < min_log_mel ? f_sp * (z) : min_log_hz * exp(logstep * ((z)-min_log_mel)))
    const double mlo = HZ2MEL(0.0), mhi = HZ2MEL(8000.0);
    double* pts = (double*)malloc(sizeof(double) * (n_mels + 2));
    for (int i = 0; i < n_mels + 2; i++) pts[i] = MEL2HZ(mlo + (mhi - mlo) * i / (n_mels + 1));
    for (int j = 0; j < n_mels; j++) {
        const double en = 2.0 / (pts[j + 2] - pts[j]);
        for (int k = 0; k < 257; k++) {
            const double fk = 8000.0 * k / 256.0;
            const double lo = (fk - pts[j]) / (pts[j + 1] - pts[j]), hi = (pts[j + 2] - fk) / (pts[j + 2] - pts[j + 1]);
            double v = lo < hi ? lo : hi;
            fb[j * 257 + k] = (float)((v > 0 ? v : 0.0) * en);
        }
    }
    free(pts);
#undef HZ2MEL
#undef MEL2HZ
}

int po_mel(const float* pcm, int n, int n_mels, float* out) {
    const int T = po_n_frames(n);
    float* fb = (float*)malloc(sizeof(float) * n_mels * 257);
    mel_filters(n_mels, fb);
    float win[512];
    for (int i = 0; i < 512; i++) {
        const int j = i - 56;  /* the 400-sample window centred in 512 */
        win[i] = (j >= 0 && j < 400) ? (float)(0.5 - 0.5 * cos(2.0 * M_PI * j / 399.0)) : 0.0f;
    }
    double cs[512], sn[512];
    for (int i = 0; i < 512; i++) {
        cs[i] = cos(2.0 * M_PI * i / 512.0);
        sn[i] = sin(2.0 * M_PI * i / 512.0);
    }
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; t++) {
        float fr[512];
        for (int i = 0; i < 512; i++) {
            const int s = t * 160 + i - 256;  /* centre padding: 256 zeros each side */
            float x = 0.0f;
            if (s >= 0 && s < n) x = pcm[s] - (s > 0 ? 0.97f * pcm[s - 1] : 0.0f);  /* pre-emphasis */
            fr[i] = x * win[i];
        }
        float pw[257];
        for (int k = 0; k < 257; k++) {
            double re = 0, im = 0;
            for (int i = 0; i < 512; i++) {
                const int ph = (k * i) & 511;
                re += fr[i] * cs[ph];
                im -= fr[i] * sn[ph];
            }
            pw[k] = (float)(re * re + im * im);
        }
        for (int j = 0; j < n_mels; j++) {
            double acc = 0;
            for (int k = 0; k < 257; k++) acc += (double)fb[j * 257 + k] * pw[k];
            out[(size_t)j * T + t] = logf((float)acc + 5.9604644775390625e-08f);  /* log(x + 2^-24) */
        }
    }
    /* per-feature normalisation over the utterance: unbiased std + 1e-5 */
    for (int j = 0; j < n_mels; j++) {
        float* r = out + (size_t)j * T;
        double mean = 0;
        for (int t = 0; t < T; t++) mean += r[t];
        mean /= T;
        double var = 0;
        for (int t = 0; t < T; t++) var += (r[t] - mean) * (r[t] - mean);
        const double sd = sqrt(var / (T > 1 ? T - 1 : 1)) + 1e-5;
        for (int t = 0; t < T; t++) r[t] = (float)((r[t] - mean) / sd);
    }
    free(fb);
    return T;
}

/* ------------------------------------------------------------------ encoder */
int po_n_enc_frames(int T) {
    for (int i = 0; i < 3; i++) T = T > 0 ? (T - 1) / 2 + 1 : 0;
    return T;
}

static void layernorm(float* x, int T, int d, const float* w, const float* b, float* out) {
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; t++) {
        const float* r = x + (size_t)t * d;
        double s = 0;
        for (int i = 0; i < d; i++) s += r[i];
        const double mean = s / d;
        double v = 0;
        for (int i = 0; i < d; i++) v += (r[i] - mean) * (r[i] - mean);
        const float rstd = (float)(1.0 / sqrt(v / d + 1e-5));
        for (int i = 0; i < d; i++) out[(size_t)t * d + i] = ((float)(r[i] - mean)) * rstd * w[i] + b[i];
    }
}

/* y[t][n] = x[t][:] . W[n][:] + b[n] */
static void linear(const float* x, int T, int K, const float* W, const float* b, int N, float* y) {
#pragma omp parallel for schedule(static) collapse(2)
    for (int t = 0; t < T; t++)
        for (int n = 0; n < N; n++) {
            const float* xr = x + (size_t)t * K;
            const float* wr = W + (size_t)n * K;
            float acc = 0.0f;
            for (int k = 0; k < K; k++) acc += xr[k] * wr[k];
            y[(size_t)t * N + n] = acc + (b ? b[n] : 0.0f);
        }
}

static inline float swish(float x) { return x / (1.0f + expf(-x)); }
static inline float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

/* NeMo ConvSubsampling(subsampling="dw_striding", factor 8): [T][F] -> [T3][d] */
static int subsample(const po_model* m, const float* mel, int T, float* out) {
    const int C = m->dm.sub_ch, F = m->dm.n_mels, d = m->dm.d;
    int Tc = T, Fc = F;
    const int T1 = (T - 1) / 2 + 1, F1 = (F - 1) / 2 + 1;
    /* conv0: Conv2d(1, C, 3, stride 2, pad 1) + ReLU; input [t][f] = mel[f][t] */
    float* a = (float*)calloc((size_t)C * T1 * F1, sizeof(float));
#pragma omp parallel for schedule(static) collapse(2)
    for (int c = 0; c < C; c++)
        for (int t = 0; t < T1; t++)
            for (int f = 0; f < F1; f++) {
                float acc = m->c0_b[c];
                for (int i = 0; i < 3; i++)
                    for (int j = 0; j < 3; j++) {
                        const int tt = 2 * t - 1 + i, ff = 2 * f - 1 + j;
                        if (tt >= 0 && tt < Tc && ff >= 0 && ff < Fc) acc += m->c0_w[c * 9 + i * 3 + j] * mel[(size_t)ff * T + tt];
                    }
                a[((size_t)c * T1 + t) * F1 + f] = acc > 0 ? acc : 0;
            }
    Tc = T1; Fc = F1;
    const float* dww[2] = {m->dw1_w, m->dw2_w};
    const float* dwb[2] = {m->dw1_b, m->dw2_b};
    const float* pww[2] = {m->pw1_w, m->pw2_w};
    const float* pwb[2] = {m->pw1_b, m->pw2_b};
    for (int s = 0; s < 2; s++) {
        const int T2 = (Tc - 1) / 2 + 1, F2 = (Fc - 1) / 2 + 1;
        float* dw = (float*)calloc((size_t)C * T2 * F2, sizeof(float));
        /* depthwise Conv2d(C, C, 3, s2, p1, groups=C) */
#pragma omp parallel for schedule(static) collapse(2)
        for (int c = 0; c < C; c++)
            for (int t = 0; t < T2; t++)
                for (int f = 0; f < F2; f++) {
                    float acc = dwb[s][c];
                    for (int i = 0; i < 3; i++)
                        for (int j = 0; j < 3; j++) {
                            const int tt = 2 * t - 1 + i, ff = 2 * f - 1 + j;
                            if (tt >= 0 && tt < Tc && ff >= 0 && ff < Fc)
                                acc += dww[s][c * 9 + i * 3 + j] * a[((size_t)c * Tc + tt) * Fc + ff];
                        }
                    dw[((size_t)c * T2 + t) * F2 + f] = acc;
                }
        /* pointwise Conv2d(C, C, 1) + ReLU */
        float* pw = (float*)calloc((size_t)C * T2 * F2, sizeof(float));
#pragma omp parallel for schedule(static) collapse(2)
        for (int o = 0; o < C; o++)
            for (int p = 0; p < T2 * F2; p++) {
                float acc = 0.0f;
                for (int c = 0; c < C; c++) acc += pww[s][(size_t)o * C + c] * dw[(size_t)c * T2 * F2 + p];
                acc += pwb[s][o];
                pw[(size_t)o * T2 * F2 + p] = acc > 0 ? acc : 0;
            }
        free(dw);
        free(a);
        a = pw;
        Tc = T2; Fc = F2;
    }
    /* flatten (b, c, t, f) -> (b, t, c * F3 + f), then Linear(C * F3, d) */
    const int K = C * Fc;
    float* flat = (float*)malloc(sizeof(float) * (size_t)Tc * K);
    for (int t = 0; t < Tc; t++)
        for (int c = 0; c < C; c++)
            for (int f = 0; f < Fc; f++) flat[(size_t)t * K + c * Fc + f] = a[((size_t)c * Tc + t) * Fc + f];
    linear(flat, Tc, K, m->sub_w, m->sub_b, d, out);
    free(flat);
    free(a);
    return Tc;
}

/* NeMo RelPositionalEncoding: rows for relative positions T-1 .. -(T-1) */
static void rel_pos(int T, int d, float* pe /* [2T-1][d] */) {
    for (int i = 0; i < 2 * T - 1; i++) {
        const double pos = (double)(T - 1 - i);
        for (int k = 0; k < d / 2; k++) {
            const double div = exp(-(2.0 * k) * log(10000.0) / d);
            pe[(size_t)i * d + 2 * k] = (float)sin(pos * div);
            pe[(size_t)i * d + 2 * k + 1] = (float)cos(pos * div);
        }
    }
}

/* NeMo RelPositionMultiHeadAttention: softmax(((q + u) k^T + rel_shift((q + v) p^T)) / sqrt(dk)) v */
static void rel_attention(const po_layer* y, const float* xn, int T, int d, int H, const float* pe, float* out) {
    const int dk = d / H, NP = 2 * T - 1;
    float *q = malloc(sizeof(float) * (size_t)T * d), *k = malloc(sizeof(float) * (size_t)T * d),
          *v = malloc(sizeof(float) * (size_t)T * d), *p = malloc(sizeof(float) * (size_t)NP * d),
          *ctx = malloc(sizeof(float) * (size_t)T * d);
    linear(xn, T, d, y->q_w, y->q_b, d, q);
    linear(xn, T, d, y->k_w, y->k_b, d, k);
    linear(xn, T, d, y->v_w, y->v_b, d, v);
    linear(pe, NP, d, y->pos_w, NULL, d, p);
    const float scale = 1.0f / sqrtf((float)dk);
#pragma omp parallel for schedule(static) collapse(2)
    for (int h = 0; h < H; h++)
        for (int i = 0; i < T; i++) {
            float* s = (float*)malloc(sizeof(float) * T);
            float mx = -INFINITY;
            for (int j = 0; j < T; j++) {
                float ac = 0.0f, bd = 0.0f;
                const float* qi = q + (size_t)i * d + h * dk;
                const float* kj = k + (size_t)j * d + h * dk;
                const float* pj = p + (size_t)(T - 1 - i + j) * d + h * dk;
                for (int e = 0; e < dk; e++) {
                    ac += (qi[e] + y->pos_u[h * dk + e]) * kj[e];
                    bd += (qi[e] + y->pos_v[h * dk + e]) * pj[e];
                }
                s[j] = (ac + bd) * scale;
                if (s[j] > mx) mx = s[j];
            }
            float l = 0.0f;
            for (int j = 0; j < T; j++) {
                s[j] = expf(s[j] - mx);
                l += s[j];
            }
            for (int e = 0; e < dk; e++) {
                float acc = 0.0f;
                for (int j = 0; j < T; j++) acc += s[j] * v[(size_t)j * d + h * dk + e];
                ctx[(size_t)i * d + h * dk + e] = acc / l;
            }
            free(s);
        }
    linear(ctx, T, d, y->o_w, y->o_b, d, out);
    free(q); free(k); free(v); free(p); free(ctx);
}

/* NeMo ConformerConvolution: pw (d -> 2d) -> GLU -> depthwise k (pad k/2) -> BatchNorm (eval,
 * eps 1e-5) -> Swish -> pw (d -> d) */
static void conv_module(const po_layer* y, const float* xn, int T, int d, int K, float* out) {
    float* a = malloc(sizeof(float) * (size_t)T * 2 * d);
    float* g = malloc(sizeof(float) * (size_t)T * d);
    float* c = malloc(sizeof(float) * (size_t)T * d);
    linear(xn, T, d, y->pw1_w, y->pw1_b, 2 * d, a);
    for (int t = 0; t < T; t++)
        for (int i = 0; i < d; i++) g[(size_t)t * d + i] = a[(size_t)t * 2 * d + i] * sigm(a[(size_t)t * 2 * d + d + i]);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < d; i++) {
        const float bs = y->bn_g[i] / sqrtf(y->bn_v[i] + 1e-5f), bt = y->bn_b[i] - y->bn_m[i] * bs;
        for (int t = 0; t < T; t++) {
            float acc = y->dw_b[i];
            for (int j = 0; j < K; j++) {
                const int tt = t - K / 2 + j;
                if (tt >= 0 && tt < T) acc += y->dw_w[i * K + j] * g[(size_t)tt * d + i];
            }
            c[(size_t)t * d + i] = swish(acc * bs + bt);
        }
    }
    linear(c, T, d, y->pw2_w, y->pw2_b, d, out);
    free(a); free(g); free(c);
}

static void ffn(const float* xn, int T, int d, int ff, const float* w1, const float* b1, const float* w2,
                const float* b2, float* out) {
    float* h = malloc(sizeof(float) * (size_t)T * ff);
    linear(xn, T, d, w1, b1, ff, h);
    for (int64_t i = 0; i < (int64_t)T * ff; i++) h[i] = swish(h[i]);
    linear(h, T, ff, w2, b2, d, out);
    free(h);
}

int po_encode(po_model* m, const float* mel, int T, float* out) {
    const po_dims* D = &m->dm;
    const int d = D->d;
    float* x = out;
    const int T3 = subsample(m, mel, T, x);
    const float xs = sqrtf((float)d);  /* RelPositionalEncoding xscale */
    for (int64_t i = 0; i < (int64_t)T3 * d; i++) x[i] *= xs;
    float* pe = malloc(sizeof(float) * (size_t)(2 * T3 - 1) * d);
    rel_pos(T3, d, pe);
    float* xn = malloc(sizeof(float) * (size_t)T3 * d);
    float* y = malloc(sizeof(float) * (size_t)T3 * d);
    for (int l = 0; l < D->n_layers; l++) {
        const po_layer* L = &m->L[l];
        /* ConformerLayer.forward */
        layernorm(x, T3, d, L->ln_ff1_w, L->ln_ff1_b, xn);
        ffn(xn, T3, d, D->ff, L->ff1_w1, L->ff1_b1, L->ff1_w2, L->ff1_b2, y);
        for (int64_t i = 0; i < (int64_t)T3 * d; i++) x[i] += 0.5f * y[i];
        layernorm(x, T3, d, L->ln_att_w, L->ln_att_b, xn);
        rel_attention(L, xn, T3, d, D->n_heads, pe, y);
        for (int64_t i = 0; i < (int64_t)T3 * d; i++) x[i] += y[i];
        layernorm(x, T3, d, L->ln_conv_w, L->ln_conv_b, xn);
        conv_module(L, xn, T3, d, D->conv_k, y);
        for (int64_t i = 0; i < (int64_t)T3 * d; i++) x[i] += y[i];
        layernorm(x, T3, d, L->ln_ff2_w, L->ln_ff2_b, xn);
        ffn(xn, T3, d, D->ff, L->ff2_w1, L->ff2_b1, L->ff2_w2, L->ff2_b2, y);
        for (int64_t i = 0; i < (int64_t)T3 * d; i++) x[i] += 0.5f * y[i];
        layernorm(x, T3, d, L->ln_out_w, L->ln_out_b, xn);
        memcpy(x, xn, sizeof(float) * (size_t)T3 * d);
    }
    free(pe); free(xn); free(y);
    return T3;
}

/* ------------------------------------------------------------------ TDT greedy */
/* one LSTM layer step (PyTorch gate order i, f, g, o) */
static void lstm_step(const float* wih, const float* whh, const float* bih, const float* bhh, int P, const float* x,
                      float* h, float* c) {
    float* gt = malloc(sizeof(float) * 4 * P);
    for (int n = 0; n < 4 * P; n++) {
        float a = bih[n] + bhh[n];
        for (int k = 0; k < P; k++) a += wih[(size_t)n * P + k] * x[k] + whh[(size_t)n * P + k] * h[k];
        gt[n] = a;
    }
    for (int j = 0; j < P; j++) {
        const float i = sigm(gt[j]), f = sigm(gt[P + j]), g = tanhf(gt[2 * P + j]), o = sigm(gt[3 * P + j]);
        c[j] = f * c[j] + i * g;
        h[j] = o * tanhf(c[j]);
    }
    free(gt);
}

/* RNNTDecoder.predict: embedding (blank row zero) -> 2-layer LSTM -> joint pred projection */
static void predict(const po_model* m, int tok, float* h /* [2][P] */, float* c, float* gp /* [J] */) {
    const int P = m->dm.pred;
    float x[4096];
    memcpy(x, m->emb + (size_t)tok * P, sizeof(float) * P);
    for (int j = 0; j < 2; j++) {
        lstm_step(m->lstm_wih[j], m->lstm_whh[j], m->lstm_bih[j], m->lstm_bhh[j], P, x, h + j * P, c + j * P);
        memcpy(x, h + j * P, sizeof(float) * P);
    }
    for (int n = 0; n < P; n++) {
        float a = m->j_pred_b[n];
        for (int k = 0; k < P; k++) a += m->j_pred_w[(size_t)n * P + k] * x[k];
        gp[n] = a;
    }
}

static int decode_core(po_model* m, const float* enc, int T3, int max_symbols, int* tokens, int* frames, float* top1,
                       float* top2, float* gmin, int cap) {
    const po_dims* D = &m->dm;
    const int P = D->pred, d = D->d, V = D->n_vocab, NO = V + 1 + D->n_dur;
    /* the joint's encoder projection of every frame, once */
    float* fe = malloc(sizeof(float) * (size_t)T3 * P);
    linear(enc, T3, d, m->j_enc_w, m->j_enc_b, P, fe);
    float h[2 * 4096], c[2 * 4096], gp[4096], hid[4096];
    memset(h, 0, sizeof(float) * 2 * P);
    memset(c, 0, sizeof(float) * 2 * P);
    predict(m, V, h, c, gp);  /* start: the blank symbol */
    float* lg = malloc(sizeof(float) * NO);
    int n = 0, t = 0, at_t = 0;
    float gacc = INFINITY;
    while (t < T3) {
        for (int k = 0; k < P; k++) {
            const float z = fe[(size_t)t * P + k] + gp[k];
            hid[k] = z > 0 ? z : 0;  /* ReLU */
        }
        for (int o = 0; o < NO; o++) {
            float a = m->j_out_b[o];
            for (int k = 0; k < P; k++) a += m->j_out_w[(size_t)o * P + k] * hid[k];
            lg[o] = a;
        }
        int tk = 0;
        float b1 = -INFINITY, b2 = -INFINITY;
        for (int o = 0; o <= V; o++) {
            if (lg[o] > b1) { b2 = b1; b1 = lg[o]; tk = o; }
            else if (lg[o] > b2) b2 = lg[o];
        }
        int dk = 0;
        float d1 = -INFINITY, d2 = -INFINITY;
        for (int o = 0; o < D->n_dur; o++) {
            const float v = lg[V + 1 + o];
            if (v > d1) { d2 = d1; d1 = v; dk = o; }
            else if (v > d2) d2 = v;
        }
        /* the closest decision (token or duration) since the previous emission */
        const float g = fminf(b1 - b2, d1 - d2);
        if (g < gacc) gacc = g;
        int skip = dk;  /* durations 0, 1, .., n_dur - 1 */
        if (tk != V) {
            if (n < cap) {
                tokens[n] = tk;
                frames[n] = t;
                if (top1) top1[n] = b1;
                if (top2) top2[n] = b2;
                if (gmin) gmin[n] = gacc;
            }
            gacc = INFINITY;
            n++;
            predict(m, tk, h, c, gp);
            at_t++;
        }
        if (skip == 0 && (tk == V || at_t >= max_symbols)) skip = 1;
        if (skip > 0) at_t = 0;
        t += skip;
    }
    if (gmin && n < cap) gmin[n] = gacc;  /* the evaluations after the last emission */
    free(lg);
    free(fe);
    return n;
}

int po_decode(po_model* m, const float* enc, int T3, int max_symbols, int* tokens, int* frames, float* top1,
              float* top2, int cap) {
    return decode_core(m, enc, T3, max_symbols, tokens, frames, top1, top2, NULL, cap);
}

int po_decode_gaps(po_model* m, const float* enc, int T3, int max_symbols, int* tokens, int* frames, float* top1,
                   float* top2, float* gmin, int cap) {
    return decode_core(m, enc, T3, max_symbols, tokens, frames, top1, top2, gmin, cap);
}
