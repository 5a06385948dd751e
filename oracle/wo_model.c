/*
 * wo_model.c -- TEST INFRASTRUCTURE (oracle).  fp32 CPU restatement of the
 * Whisper encoder / cross-KV / decoder / greedy loop that whisper.cpp's
 * whisper_full() runs for TranscriptionManager::transcribe
 * (/root/reference/src-tauri/src/managers/transcription.rs:494-503 ->
 * transcribe-rs WhisperEngine::transcribe_samples -> whisper-rs -> whisper.cpp,
 * none vendored; restated from upstream whisper.cpp ~v1.7.x):
 *   whisper_build_graph_conv     conv1(k3,p1)+b, GELU, conv2(k3,s2,p1)+b, GELU, + e_pe
 *   whisper_build_graph_encoder  pre-LN MHA (K has no bias, 1/sqrt(64) scale,
 *                                 no mask) + pre-LN MLP(GELU), ln_post
 *   whisper_build_graph_cross    K = enc.W_k, V = enc.W_v + b_v per decoder layer
 *   whisper_build_graph_decoder  tok_emb[tok] + pos[p]; causal self-attn with
 *                                 KV cache, cross-attn, MLP; ln; logits = x.E^T
 *   whisper_process_logits       suppress blank (first step), <|notimestamps|>,
 *                                 timestamps, sot/nosp/solm/translate/transcribe/
 *                                 prev, language tokens; greedy argmax
 * LayerNorm sums in double like ggml_compute_forward_norm_f32; eps 1e-5.
 * GELU: tanh form (ggml) or erf (HF) by switch.
 *
 * Synthetic weights: counter-based splitmix64 PRNG, power-of-two scales (so
 * every generated value is exact in fp32 and identical on the GPU); matrices
 * optionally rounded to bf16 (RNE) to match the bf16 engine's storage.
 * The tensor table below is the contract shared with spittle_amd/csrc/weights.cpp.
 */
#include "whisper_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ PRNG */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
/* uniform in [-1, 1) with 24 significant bits, exact in fp32 */
static inline float urand(uint64_t seed, uint32_t tid, uint64_t i) {
    uint64_t x = i + ((uint64_t)tid << 32) + seed * 0xD1B54A32D192ED03ULL;
    uint64_t z = mix64(x);
    return (float)(uint32_t)(z >> 40) * (1.0f / 8388608.0f) - 1.0f;
}
static inline float bf16_round(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
    memcpy(&f, &u, 4);
    return f;
}
static int pow2_exp_for_fanin(int K) {
    return (int)floor(log2(sqrt(3.0 / (double)K)) + 0.5);
}

enum { K_MAT = 0, K_BIAS, K_LNW, K_LNB, K_TOK, K_DPOS, K_EPOS };

typedef struct {
    float *ln1_w, *ln1_b, *q_w, *q_b, *k_w, *v_w, *v_b, *o_w, *o_b, *ln2_w, *ln2_b,
          *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} enc_layer;
typedef struct {
    float *ln1_w, *ln1_b, *sq_w, *sq_b, *sk_w, *sv_w, *sv_b, *so_w, *so_b,
          *ln2_w, *ln2_b, *cq_w, *cq_b, *ck_w, *cv_w, *cv_b, *co_w, *co_b,
          *ln3_w, *ln3_b, *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} dec_layer;

typedef struct { int tid; int kind; int fanin; int64_t numel; float** slot; } tinfo;

struct wo_model {
    wo_dims dm;
    uint64_t seed;
    int wdtype;
    float *conv1_w, *conv1_b, *conv2_w, *conv2_b, *enc_pos, *lnp_w, *lnp_b;
    float *tok_emb, *dec_pos, *lnf_w, *lnf_b;
    enc_layer* enc;
    dec_layer* dec;
    int n_t;
    tinfo* t;
};

/* tensor table: (tid, kind, fan-in, numel).  Ids:
 *   encoder stem 1..6, encoder layer l: 100 + 32 l + {0..14},
 *   decoder globals 10..13, decoder layer l: 5000 + 32 l + {0..23}. */
static void add_t(wo_model* m, int tid, int kind, int fanin, int64_t numel, float** slot) {
    tinfo* ti = &m->t[m->n_t++];
    ti->tid = tid; ti->kind = kind; ti->fanin = fanin; ti->numel = numel; ti->slot = slot;
}

static void build_table(wo_model* m) {
    const int d = m->dm.d, nm = m->dm.n_mels, V = m->dm.n_vocab;
    const int64_t dd = (int64_t)d * d;
    m->t = (tinfo*)calloc(16 + 15 * m->dm.n_enc + 24 * m->dm.n_dec, sizeof(tinfo));
    add_t(m, 1, K_MAT, nm * 3, (int64_t)d * nm * 3, &m->conv1_w);
    add_t(m, 2, K_BIAS, 0, d, &m->conv1_b);
    add_t(m, 3, K_MAT, d * 3, dd * 3, &m->conv2_w);
    add_t(m, 4, K_BIAS, 0, d, &m->conv2_b);
    add_t(m, 5, K_LNW, 0, d, &m->lnp_w);
    add_t(m, 6, K_LNB, 0, d, &m->lnp_b);
    add_t(m, 7, K_EPOS, 0, (int64_t)m->dm.n_audio_ctx * d, &m->enc_pos);
    for (int l = 0; l < m->dm.n_enc; l++) {
        enc_layer* L = &m->enc[l];
        int b = 100 + 32 * l;
        add_t(m, b + 0, K_LNW, 0, d, &L->ln1_w);
        add_t(m, b + 1, K_LNB, 0, d, &L->ln1_b);
        add_t(m, b + 2, K_MAT, d, dd, &L->q_w);
        add_t(m, b + 3, K_BIAS, 0, d, &L->q_b);
        add_t(m, b + 4, K_MAT, d, dd, &L->k_w);
        add_t(m, b + 5, K_MAT, d, dd, &L->v_w);
        add_t(m, b + 6, K_BIAS, 0, d, &L->v_b);
        add_t(m, b + 7, K_MAT, d, dd, &L->o_w);
        add_t(m, b + 8, K_BIAS, 0, d, &L->o_b);
        add_t(m, b + 9, K_LNW, 0, d, &L->ln2_w);
        add_t(m, b + 10, K_LNB, 0, d, &L->ln2_b);
        add_t(m, b + 11, K_MAT, d, dd * 4, &L->fc1_w);
        add_t(m, b + 12, K_BIAS, 0, 4 * d, &L->fc1_b);
        add_t(m, b + 13, K_MAT, 4 * d, dd * 4, &L->fc2_w);
        add_t(m, b + 14, K_BIAS, 0, d, &L->fc2_b);
    }
    add_t(m, 10, K_TOK, 0, (int64_t)V * d, &m->tok_emb);
    add_t(m, 11, K_DPOS, 0, (int64_t)m->dm.n_text_ctx * d, &m->dec_pos);
    add_t(m, 12, K_LNW, 0, d, &m->lnf_w);
    add_t(m, 13, K_LNB, 0, d, &m->lnf_b);
    for (int l = 0; l < m->dm.n_dec; l++) {
        dec_layer* L = &m->dec[l];
        int b = 5000 + 32 * l;
        add_t(m, b + 0, K_LNW, 0, d, &L->ln1_w);
        add_t(m, b + 1, K_LNB, 0, d, &L->ln1_b);
        add_t(m, b + 2, K_MAT, d, dd, &L->sq_w);
        add_t(m, b + 3, K_BIAS, 0, d, &L->sq_b);
        add_t(m, b + 4, K_MAT, d, dd, &L->sk_w);
        add_t(m, b + 5, K_MAT, d, dd, &L->sv_w);
        add_t(m, b + 6, K_BIAS, 0, d, &L->sv_b);
        add_t(m, b + 7, K_MAT, d, dd, &L->so_w);
        add_t(m, b + 8, K_BIAS, 0, d, &L->so_b);
        add_t(m, b + 9, K_LNW, 0, d, &L->ln2_w);
        add_t(m, b + 10, K_LNB, 0, d, &L->ln2_b);
        add_t(m, b + 11, K_MAT, d, dd, &L->cq_w);
        add_t(m, b + 12, K_BIAS, 0, d, &L->cq_b);
        add_t(m, b + 13, K_MAT, d, dd, &L->ck_w);
        add_t(m, b + 14, K_MAT, d, dd, &L->cv_w);
        add_t(m, b + 15, K_BIAS, 0, d, &L->cv_b);
        add_t(m, b + 16, K_MAT, d, dd, &L->co_w);
        add_t(m, b + 17, K_BIAS, 0, d, &L->co_b);
        add_t(m, b + 18, K_LNW, 0, d, &L->ln3_w);
        add_t(m, b + 19, K_LNB, 0, d, &L->ln3_b);
        add_t(m, b + 20, K_MAT, d, dd * 4, &L->fc1_w);
        add_t(m, b + 21, K_BIAS, 0, 4 * d, &L->fc1_b);
        add_t(m, b + 22, K_MAT, 4 * d, dd * 4, &L->fc2_w);
        add_t(m, b + 23, K_BIAS, 0, d, &L->fc2_b);
    }
}

/* encoder positional embedding: whisper sinusoids(1500, d), computed in double */
static void fill_sinusoids(float* out, int T, int d) {
    const int half = d / 2;
    const double inc = log(10000.0) / (double)(half - 1);
    for (int t = 0; t < T; t++)
        for (int i = 0; i < half; i++) {
            double st = (double)t * exp(-inc * (double)i);
            out[(size_t)t * d + i] = (float)sin(st);
            out[(size_t)t * d + half + i] = (float)cos(st);
        }
}

static void gen_tensor(const wo_model* m, const tinfo* ti, float* dst) {
    const uint64_t seed = m->seed;
    if (ti->kind == K_EPOS) { fill_sinusoids(dst, m->dm.n_audio_ctx, m->dm.d); return; }
    float scale = 1.0f;
    switch (ti->kind) {
        case K_MAT: scale = ldexpf(1.0f, pow2_exp_for_fanin(ti->fanin)); break;
        case K_BIAS: scale = ldexpf(1.0f, -5); break;
        case K_LNW: scale = ldexpf(1.0f, -3); break;
        case K_LNB: scale = ldexpf(1.0f, -4); break;
        case K_TOK: scale = ldexpf(1.0f, -2); break;
        case K_DPOS: scale = ldexpf(1.0f, 0); break;
    }
    const int round = (m->wdtype == WO_W_BF16) && (ti->kind == K_MAT || ti->kind == K_TOK);
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < ti->numel; i++) {
        float v = urand(seed, (uint32_t)ti->tid, (uint64_t)i) * scale;
        if (ti->kind == K_LNW) v = 1.0f + v;
        if (round) v = bf16_round(v);
        dst[i] = v;
    }
}

wo_model* wo_model_new(const wo_dims* dm, uint64_t seed, int wdtype) {
    wo_model* m = (wo_model*)calloc(1, sizeof(wo_model));
    m->dm = *dm;
    m->seed = seed;
    m->wdtype = wdtype;
    m->enc = (enc_layer*)calloc(dm->n_enc > 0 ? dm->n_enc : 1, sizeof(enc_layer));
    m->dec = (dec_layer*)calloc(dm->n_dec > 0 ? dm->n_dec : 1, sizeof(dec_layer));
    build_table(m);
    for (int i = 0; i < m->n_t; i++) {
        tinfo* ti = &m->t[i];
        *ti->slot = (float*)malloc(sizeof(float) * ti->numel);
        gen_tensor(m, ti, *ti->slot);
    }
    return m;
}

void wo_model_free(wo_model* m) {
    if (!m) return;
    for (int i = 0; i < m->n_t; i++) free(*m->t[i].slot);
    free(m->t);
    free(m->enc);
    free(m->dec);
    free(m);
}

int wo_tensor_count(const wo_model* m) { return m->n_t; }
int wo_tensor_info(const wo_model* m, int i, int* tid, int64_t* numel, const float** data) {
    if (i < 0 || i >= m->n_t) return -1;
    *tid = m->t[i].tid;
    *numel = m->t[i].numel;
    *data = *m->t[i].slot;
    return 0;
}

int wo_tensor_set(wo_model* m, int tid, const float* data, int64_t numel) {
    for (int i = 0; i < m->n_t; i++)
        if (m->t[i].tid == tid) {
            if (m->t[i].numel != numel) return -2;
            memcpy(*m->t[i].slot, data, sizeof(float) * (size_t)numel);
            return 0;
        }
    return -1;
}

void wo_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ---------------------------------------------------------- primitives */
typedef float v8f __attribute__((vector_size(32), aligned(4)));

static inline float hsum8(v8f v) {
    return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

/* C[m][n] = sum_k A[m][k] W[n][k] (+ bias[n]); fp32 */
static void gemm_nt(int M, int N, int K, const float* A, int lda, const float* W, int ldw,
                    float* C, int ldc, const float* bias) {
    const int NB = 64;
    const int nblk = (N + NB - 1) / NB;
    const int K8 = K & ~7;
    #pragma omp parallel for schedule(dynamic, 1)
    for (int bi = 0; bi < nblk; bi++) {
        const int n0 = bi * NB, n1 = n0 + NB < N ? n0 + NB : N;
        int m = 0;
        for (; m + 4 <= M; m += 4) {
            int n = n0;
            for (; n + 4 <= n1; n += 4) {
                v8f acc[4][4];
                memset(acc, 0, sizeof acc);
                const float* a0 = A + (size_t)m * lda;
                const float* w0 = W + (size_t)n * ldw;
                for (int k = 0; k < K8; k += 8) {
                    v8f a[4], w[4];
                    for (int i = 0; i < 4; i++) a[i] = *(const v8f*)(a0 + (size_t)i * lda + k);
                    for (int j = 0; j < 4; j++) w[j] = *(const v8f*)(w0 + (size_t)j * ldw + k);
                    for (int i = 0; i < 4; i++)
                        for (int j = 0; j < 4; j++) acc[i][j] += a[i] * w[j];
                }
                for (int i = 0; i < 4; i++)
                    for (int j = 0; j < 4; j++) {
                        float s = hsum8(acc[i][j]);
                        for (int k = K8; k < K; k++) s += a0[(size_t)i * lda + k] * w0[(size_t)j * ldw + k];
                        C[(size_t)(m + i) * ldc + n + j] = s + (bias ? bias[n + j] : 0.0f);
                    }
            }
            for (; n < n1; n++)
                for (int i = 0; i < 4; i++) {
                    const float* a = A + (size_t)(m + i) * lda;
                    const float* w = W + (size_t)n * ldw;
                    v8f acc = {0};
                    for (int k = 0; k < K8; k += 8) acc += *(const v8f*)(a + k) * *(const v8f*)(w + k);
                    float s = hsum8(acc);
                    for (int k = K8; k < K; k++) s += a[k] * w[k];
                    C[(size_t)(m + i) * ldc + n] = s + (bias ? bias[n] : 0.0f);
                }
        }
        for (; m < M; m++) {
            const float* a = A + (size_t)m * lda;
            int n = n0;
            for (; n + 4 <= n1; n += 4) {
                v8f acc[4] = {{0}, {0}, {0}, {0}};
                for (int k = 0; k < K8; k += 8) {
                    v8f av = *(const v8f*)(a + k);
                    for (int j = 0; j < 4; j++) acc[j] += av * *(const v8f*)(W + (size_t)(n + j) * ldw + k);
                }
                for (int j = 0; j < 4; j++) {
                    float s = hsum8(acc[j]);
                    for (int k = K8; k < K; k++) s += a[k] * W[(size_t)(n + j) * ldw + k];
                    C[(size_t)m * ldc + n + j] = s + (bias ? bias[n + j] : 0.0f);
                }
            }
            for (; n < n1; n++) {
                const float* w = W + (size_t)n * ldw;
                v8f acc = {0};
                for (int k = 0; k < K8; k += 8) acc += *(const v8f*)(a + k) * *(const v8f*)(w + k);
                float s = hsum8(acc);
                for (int k = K8; k < K; k++) s += a[k] * w[k];
                C[(size_t)m * ldc + n] = s + (bias ? bias[n] : 0.0f);
            }
        }
    }
}

/* ggml_compute_forward_norm_f32 (double sums) then *w + b */
static void layernorm(int M, int d, const float* x, const float* w, const float* b, float* y) {
    #pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++) {
        const float* xr = x + (size_t)m * d;
        float* yr = y + (size_t)m * d;
        double sum = 0.0;
        for (int i = 0; i < d; i++) sum += (double)xr[i];
        const float mean = (float)(sum / d);
        double sum2 = 0.0;
        for (int i = 0; i < d; i++) {
            float v = xr[i] - mean;
            sum2 += (double)(v * v);
        }
        const float var = (float)(sum2 / d);
        const float scale = 1.0f / sqrtf(var + 1e-5f);
        for (int i = 0; i < d; i++) yr[i] = (xr[i] - mean) * scale * w[i] + b[i];
    }
}

static inline float gelu1(float x, int mode) {
    if (mode == WO_GELU_ERF) return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
    const float c = 0.7978845608028654f; /* sqrt(2/pi) */
    return 0.5f * x * (1.0f + tanhf(c * (x + 0.044715f * x * x * x)));
}
static void gelu_inplace(size_t n, float* x, int mode) {
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) x[i] = gelu1(x[i], mode);
}

static void add_inplace(size_t n, float* y, const float* x) {
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) y[i] += x[i];
}

/* multi-head attention: O[t][h*64+e] = softmax(q.k / 8) v.
 * q rows at Q + t*ldq + h*64; k/v rows at K + s*ldk + h*64.
 * causal: query t (absolute position qpos0 + t) sees keys s <= qpos0 + t. */
static void attention(int Tq, int Tk, int H, const float* Q, int ldq, const float* K, int ldk,
                      const float* V, int ldv, float* O, int ldo, int causal, int qpos0) {
    #pragma omp parallel
    {
        float* p = (float*)malloc(sizeof(float) * (Tk > 0 ? Tk : 1));
        #pragma omp for collapse(2) schedule(static)
        for (int h = 0; h < H; h++)
            for (int t = 0; t < Tq; t++) {
                const float* q = Q + (size_t)t * ldq + h * 64;
                const int nk = causal ? (qpos0 + t + 1 < Tk ? qpos0 + t + 1 : Tk) : Tk;
                float mx = -INFINITY;
                for (int s = 0; s < nk; s++) {
                    const float* k = K + (size_t)s * ldk + h * 64;
                    v8f acc = {0};
                    for (int e = 0; e < 64; e += 8) acc += *(const v8f*)(q + e) * *(const v8f*)(k + e);
                    float sc = hsum8(acc) * 0.125f;
                    p[s] = sc;
                    if (sc > mx) mx = sc;
                }
                double sum = 0.0;
                for (int s = 0; s < nk; s++) {
                    p[s] = expf(p[s] - mx);
                    sum += p[s];
                }
                const float inv = (float)(1.0 / sum);
                float o[64];
                for (int e = 0; e < 64; e++) o[e] = 0.0f;
                for (int s = 0; s < nk; s++) {
                    const float* v = V + (size_t)s * ldv + h * 64;
                    const float ps = p[s];
                    for (int e = 0; e < 64; e++) o[e] += ps * v[e];
                }
                float* orow = O + (size_t)t * ldo + h * 64;
                for (int e = 0; e < 64; e++) orow[e] = o[e] * inv;
            }
        free(p);
    }
}

/* ------------------------------------------------------------- encoder */
int wo_encode(const wo_model* m, const float* mel, int gelu_mode, float* out) {
    const int d = m->dm.d, nm = m->dm.n_mels, T2 = m->dm.n_audio_ctx, T1 = 2 * T2, H = m->dm.n_head;
    /* conv1: im2col X1[t][c*3+j] = mel[c][t-1+j] */
    float* X1 = (float*)calloc((size_t)T1 * nm * 3, sizeof(float));
    #pragma omp parallel for schedule(static)
    for (int t = 0; t < T1; t++)
        for (int c = 0; c < nm; c++)
            for (int j = 0; j < 3; j++) {
                int s = t - 1 + j;
                X1[(size_t)t * nm * 3 + c * 3 + j] = (s >= 0 && s < T1) ? mel[(size_t)c * T1 + s] : 0.0f;
            }
    float* Y1 = (float*)malloc(sizeof(float) * (size_t)T1 * d);
    gemm_nt(T1, d, nm * 3, X1, nm * 3, m->conv1_w, nm * 3, Y1, d, m->conv1_b);
    gelu_inplace((size_t)T1 * d, Y1, gelu_mode);
    free(X1);
    /* conv2 stride 2: X2[t][c*3+j] = Y1[2t-1+j][c] */
    float* X2 = (float*)malloc(sizeof(float) * (size_t)T2 * d * 3);
    #pragma omp parallel for schedule(static)
    for (int t = 0; t < T2; t++)
        for (int c = 0; c < d; c++)
            for (int j = 0; j < 3; j++) {
                int s = 2 * t - 1 + j;
                X2[(size_t)t * d * 3 + c * 3 + j] = (s >= 0 && s < T1) ? Y1[(size_t)s * d + c] : 0.0f;
            }
    float* x = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    gemm_nt(T2, d, d * 3, X2, d * 3, m->conv2_w, d * 3, x, d, m->conv2_b);
    gelu_inplace((size_t)T2 * d, x, gelu_mode);
    add_inplace((size_t)T2 * d, x, m->enc_pos);
    free(X2);
    free(Y1);

    float* h = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    float* q = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    float* k = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    float* v = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    float* a = (float*)malloc(sizeof(float) * (size_t)T2 * d);
    float* f = (float*)malloc(sizeof(float) * (size_t)T2 * d * 4);
    for (int l = 0; l < m->dm.n_enc; l++) {
        const enc_layer* L = &m->enc[l];
        layernorm(T2, d, x, L->ln1_w, L->ln1_b, h);
        gemm_nt(T2, d, d, h, d, L->q_w, d, q, d, L->q_b);
        gemm_nt(T2, d, d, h, d, L->k_w, d, k, d, NULL);
        gemm_nt(T2, d, d, h, d, L->v_w, d, v, d, L->v_b);
        attention(T2, T2, H, q, d, k, d, v, d, a, d, 0, 0);
        gemm_nt(T2, d, d, a, d, L->o_w, d, h, d, L->o_b);
        add_inplace((size_t)T2 * d, x, h);
        layernorm(T2, d, x, L->ln2_w, L->ln2_b, h);
        gemm_nt(T2, 4 * d, d, h, d, L->fc1_w, d, f, 4 * d, L->fc1_b);
        gelu_inplace((size_t)T2 * d * 4, f, gelu_mode);
        gemm_nt(T2, d, 4 * d, f, 4 * d, L->fc2_w, 4 * d, h, d, L->fc2_b);
        add_inplace((size_t)T2 * d, x, h);
    }
    layernorm(T2, d, x, m->lnp_w, m->lnp_b, out);
    free(h); free(q); free(k); free(v); free(a); free(f); free(x);
    return 0;
}

/* ------------------------------------------------------------- decoder */
void wo_special_tokens(int n_vocab, int32_t o[10]) {
    /* whisper_vocab defaults + the multilingual shift of whisper_model_load */
    int eot = 50256, sot = 50257, translate = 50357, transcribe = 50358, solm = 50359,
        prev = 50360, nosp = 50361, not_ = 50362, beg = 50363;
    const int multi = n_vocab >= 51865;
    const int n_langs = n_vocab - 51765 - (multi ? 1 : 0);
    if (multi) {
        eot++; sot++;
        const int dt = n_langs - 98;
        translate += dt; transcribe += dt; solm += dt; prev += dt; nosp += dt; not_ += dt; beg += dt;
    }
    o[0] = eot; o[1] = sot; o[2] = translate; o[3] = transcribe; o[4] = solm;
    o[5] = prev; o[6] = nosp; o[7] = not_; o[8] = beg; o[9] = multi ? n_langs : 0;
}

typedef struct {
    float *ks, *vs;   /* self cache [L][n_text_ctx][d] */
    float *kc, *vc;   /* cross [L][1500][d] */
    float *x, *h, *q, *k, *v, *a, *f, *logits;
    int cap_rows;
} dec_state;

static void dec_state_init(const wo_model* m, const float* enc, dec_state* s, int cap_rows) {
    const int d = m->dm.d, L = m->dm.n_dec, T = m->dm.n_audio_ctx, C = m->dm.n_text_ctx;
    s->ks = (float*)calloc((size_t)L * C * d, sizeof(float));
    s->vs = (float*)calloc((size_t)L * C * d, sizeof(float));
    s->kc = (float*)malloc(sizeof(float) * (size_t)L * T * d);
    s->vc = (float*)malloc(sizeof(float) * (size_t)L * T * d);
    for (int l = 0; l < L; l++) {
        gemm_nt(T, d, d, enc, d, m->dec[l].ck_w, d, s->kc + (size_t)l * T * d, d, NULL);
        gemm_nt(T, d, d, enc, d, m->dec[l].cv_w, d, s->vc + (size_t)l * T * d, d, m->dec[l].cv_b);
    }
    s->cap_rows = cap_rows;
    s->x = (float*)malloc(sizeof(float) * cap_rows * d);
    s->h = (float*)malloc(sizeof(float) * cap_rows * d);
    s->q = (float*)malloc(sizeof(float) * cap_rows * d);
    s->k = (float*)malloc(sizeof(float) * cap_rows * d);
    s->v = (float*)malloc(sizeof(float) * cap_rows * d);
    s->a = (float*)malloc(sizeof(float) * cap_rows * d);
    s->f = (float*)malloc(sizeof(float) * cap_rows * d * 4);
    s->logits = (float*)malloc(sizeof(float) * m->dm.n_vocab);
}
static void dec_state_free(dec_state* s) {
    free(s->ks); free(s->vs); free(s->kc); free(s->vc);
    free(s->x); free(s->h); free(s->q); free(s->k); free(s->v); free(s->a); free(s->f);
    free(s->logits);
}

/* run n tokens at positions pos0.. through the decoder; logits of the last row */
static void dec_forward(const wo_model* m, dec_state* s, const int32_t* toks, int n, int pos0,
                        int gelu_mode) {
    const int d = m->dm.d, C = m->dm.n_text_ctx, T = m->dm.n_audio_ctx, H = m->dm.n_head;
    for (int r = 0; r < n; r++)
        for (int i = 0; i < d; i++)
            s->x[(size_t)r * d + i] = m->tok_emb[(size_t)toks[r] * d + i] + m->dec_pos[(size_t)(pos0 + r) * d + i];
    for (int l = 0; l < m->dm.n_dec; l++) {
        const dec_layer* L = &m->dec[l];
        float* ks = s->ks + (size_t)l * C * d;
        float* vs = s->vs + (size_t)l * C * d;
        layernorm(n, d, s->x, L->ln1_w, L->ln1_b, s->h);
        gemm_nt(n, d, d, s->h, d, L->sq_w, d, s->q, d, L->sq_b);
        gemm_nt(n, d, d, s->h, d, L->sk_w, d, ks + (size_t)pos0 * d, d, NULL);
        gemm_nt(n, d, d, s->h, d, L->sv_w, d, vs + (size_t)pos0 * d, d, L->sv_b);
        attention(n, pos0 + n, H, s->q, d, ks, d, vs, d, s->a, d, 1, pos0);
        gemm_nt(n, d, d, s->a, d, L->so_w, d, s->h, d, L->so_b);
        add_inplace((size_t)n * d, s->x, s->h);
        layernorm(n, d, s->x, L->ln2_w, L->ln2_b, s->h);
        gemm_nt(n, d, d, s->h, d, L->cq_w, d, s->q, d, L->cq_b);
        attention(n, T, H, s->q, d, s->kc + (size_t)l * T * d, d, s->vc + (size_t)l * T * d, d,
                  s->a, d, 0, 0);
        gemm_nt(n, d, d, s->a, d, L->co_w, d, s->h, d, L->co_b);
        add_inplace((size_t)n * d, s->x, s->h);
        layernorm(n, d, s->x, L->ln3_w, L->ln3_b, s->h);
        gemm_nt(n, 4 * d, d, s->h, d, L->fc1_w, d, s->f, 4 * d, L->fc1_b);
        gelu_inplace((size_t)n * 4 * d, s->f, gelu_mode);
        gemm_nt(n, d, 4 * d, s->f, 4 * d, L->fc2_w, 4 * d, s->h, d, L->fc2_b);
        add_inplace((size_t)n * d, s->x, s->h);
    }
    layernorm(1, d, s->x + (size_t)(n - 1) * d, m->lnf_w, m->lnf_b, s->h);
    gemm_nt(1, m->dm.n_vocab, d, s->h, d, m->tok_emb, d, s->logits, m->dm.n_vocab, NULL);
}

int wo_decode_logits(const wo_model* m, const float* enc, const int32_t* toks, int n_toks,
                     int gelu_mode, float* logits) {
    if (n_toks <= 0 || n_toks > m->dm.n_text_ctx) return -1;
    dec_state s;
    dec_state_init(m, enc, &s, n_toks);
    dec_forward(m, &s, toks, n_toks, 0, gelu_mode);
    memcpy(logits, s.logits, sizeof(float) * m->dm.n_vocab);
    dec_state_free(&s);
    return 0;
}

/* whisper.cpp whisper_lang_auto_detect_with_state, offset_ms = 0: decode [sot] at n_past 0,
 * take the logits of the n_langs language tokens (sot + 1 + i), sort them descending and
 * return the first; probabilities are the softmax over the language logits only. */
int wo_lang_detect(const wo_model* m, const float* enc, int gelu_mode, float* probs) {
    int32_t sp[10];
    wo_special_tokens(m->dm.n_vocab, sp);
    const int n_langs = sp[9];
    if (n_langs <= 0) return -1;
    dec_state s;
    dec_state_init(m, enc, &s, 1);
    const int32_t sot = sp[1];
    dec_forward(m, &s, &sot, 1, 0, gelu_mode);
    int best = 0;
    float bmax = -INFINITY;
    for (int i = 0; i < n_langs; i++) {
        const float v = s.logits[sot + 1 + i];
        if (v > bmax) { bmax = v; best = i; }
    }
    if (probs) {
        double sum = 0.0;
        for (int i = 0; i < n_langs; i++) {
            probs[i] = expf(s.logits[sot + 1 + i] - bmax);
            sum += probs[i];
        }
        for (int i = 0; i < n_langs; i++) probs[i] = (float)(probs[i] / sum);
    }
    dec_state_free(&s);
    return best;
}

/* whisper_process_logits, greedy / no-timestamp subset */
static void suppress(const wo_model* m, float* lg, int is_initial, uint32_t flags) {
    int32_t sp[10];
    wo_special_tokens(m->dm.n_vocab, sp);
    const int V = m->dm.n_vocab;
    if ((flags & WO_SUPPRESS_BLANK) && is_initial) {
        lg[sp[0]] = -INFINITY;
        lg[220] = -INFINITY; /* " " */
    }
    lg[sp[7]] = -INFINITY;
    if (flags & WO_NO_TIMESTAMPS)
        for (int i = sp[8]; i < V; i++) lg[i] = -INFINITY;
    lg[sp[1]] = -INFINITY;
    lg[sp[6]] = -INFINITY;
    lg[sp[4]] = -INFINITY;
    lg[sp[2]] = -INFINITY;
    lg[sp[3]] = -INFINITY;
    lg[sp[5]] = -INFINITY;
    for (int i = 0; i < sp[9]; i++) lg[sp[1] + 1 + i] = -INFINITY;
}

int wo_decode(const wo_model* m, const float* enc, const int32_t* prompt, int n_prompt,
              int n_steps, uint32_t flags, int gelu_mode, const int32_t* forced,
              int32_t* tokens, float* top1, float* top2) {
    if (n_prompt <= 0 || n_prompt + n_steps > m->dm.n_text_ctx + 1) return -1;
    int32_t sp[10];
    wo_special_tokens(m->dm.n_vocab, sp);
    dec_state s;
    dec_state_init(m, enc, &s, n_prompt);
    const int V = m->dm.n_vocab;
    int pos = 0, done = 0, produced = 0;
    int32_t feed = 0;
    for (int step = 0; step < n_steps; step++) {
        if (done) { tokens[step] = -1; top1[step] = top2[step] = -INFINITY; continue; }
        if (step == 0) { dec_forward(m, &s, prompt, n_prompt, 0, gelu_mode); pos = n_prompt; }
        else { dec_forward(m, &s, &feed, 1, pos, gelu_mode); pos++; }
        suppress(m, s.logits, step == 0, flags);
        int best = 0;
        float b1 = -INFINITY, b2 = -INFINITY;
        for (int i = 0; i < V; i++) {
            float v = s.logits[i];
            if (v > b1) { b2 = b1; b1 = v; best = i; }
            else if (v > b2) b2 = v;
        }
        tokens[step] = best;
        top1[step] = b1;
        top2[step] = b2;
        produced++;
        feed = forced ? forced[step] : best;
        if (!(flags & WO_IGNORE_EOT) && best == sp[0]) done = 1;
        if (pos >= m->dm.n_text_ctx) done = 1;
    }
    dec_state_free(&s);
    return produced;
}
