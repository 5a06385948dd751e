/* capi_smoke.c -- the exact call sequence the Rust binding (rust/spittle-hip) performs, in C,
 * through include/spittle_hip.h and libspittle_hip.so:
 *   load_model          spt_default_model_params + spt_ctx_create   (transcription.rs:261-276)
 *   transcribe_samples  spt_default_infer_params + language/initial_prompt + spt_transcribe
 *                       -> read text / segments -> spt_result_free    (transcription.rs:494-503)
 *   unload_model        spt_ctx_destroy                               (transcription.rs:175-208)
 * then the same again (the idle watcher unloads, the next dictation reloads), and the error
 * paths the binding maps to Err(..).  With a third argument, the Parakeet sequence of
 * HipParakeetEngine on that model directory (the catalog's int8 ONNX export layout):
 *   load_model_with_params(&path, ParakeetModelParams::int8())  spt_parakeet_create(dir)
 *                                                                (transcription.rs:278-297)
 *   transcribe_samples(.., Segment)   spt_parakeet_transcribe    (transcription.rs:505-513)
 * (with --link-only: the host-only loader, spt_parakeet_onnx_open, no device).
 * Exit 0 = every step behaved. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spittle_hip.h"

#define CHECK(c, msg)                                                       \
    do {                                                                    \
        if (!(c)) {                                                         \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, msg);   \
            return 1;                                                       \
        }                                                                   \
    } while (0)

static int one_session(const char* spec, const float* pcm, size_t n) {
    spt_model_params mp;
    spt_default_model_params(&mp);
    mp.dtype = SPT_DTYPE_F32;
    mp.max_batch = 5; /* whisper_full's best_of decoders fit one call */
    spt_ctx* ctx = NULL;
    char err[512] = {0};
    spt_status st = spt_ctx_create(spec, &mp, &ctx, err, sizeof err);
    if (st != SPT_OK) fprintf(stderr, "create: %s\n", err);
    CHECK(st == SPT_OK && ctx, "spt_ctx_create");

    spt_model_info info;
    CHECK(spt_ctx_info(ctx, &info) == SPT_OK && info.n_audio_ctx == 1500, "spt_ctx_info");

    /* the app's params: whisper_full defaults + language + (for ggml models) initial_prompt */
    spt_infer_params ip;
    spt_default_infer_params(&ip);
    ip.language = "en";
    ip.max_new_tokens = 16;
    spt_result* r = NULL;
    st = spt_transcribe(ctx, pcm, n, &ip, &r);
    if (st != SPT_OK) fprintf(stderr, "transcribe: %s\n", spt_last_error(ctx));
    CHECK(st == SPT_OK && r && r->text, "spt_transcribe (whisper_full defaults)");
    CHECK(r->n_windows >= 1 && r->n_tokens >= 0, "result fields");
    for (int i = 0; i < r->n_segments; ++i)
        CHECK(r->segments[i].text && r->segments[i].t1 >= r->segments[i].t0, "segment");
    printf("whisper_full: %d tokens, %d segments, text \"%.60s\"\n", r->n_tokens, r->n_segments, r->text);
    spt_result_free(r);

    /* an initial_prompt needs a vocabulary: a synthetic model reports it, it does not crash */
    ip.initial_prompt = "Technical dictation. Common terms: Kubernetes";
    r = NULL;
    st = spt_transcribe(ctx, pcm, n, &ip, &r);
    CHECK(st == SPT_ERR_UNSUPPORTED && r == NULL && strlen(spt_last_error(ctx)) > 0, "initial_prompt without vocab");
    ip.initial_prompt = NULL;

    /* empty audio: "" without device work */
    r = NULL;
    CHECK(spt_transcribe(ctx, pcm, 0, &ip, &r) == SPT_OK && r && r->text[0] == 0, "empty audio");
    spt_result_free(r);

    /* the benchmark protocol (device-resident greedy, no timestamps) */
    ip.flags = SPT_SUPPRESS_BLANK | SPT_NO_TIMESTAMPS | SPT_IGNORE_EOT;
    ip.temperature_inc = 0.0f;
    ip.max_new_tokens = 8;
    r = NULL;
    CHECK(spt_transcribe(ctx, pcm, n, &ip, &r) == SPT_OK && r->n_tokens == 8, "fast path");
    spt_result_free(r);

    /* bad arguments are errors, not crashes */
    CHECK(spt_transcribe(ctx, NULL, 10, &ip, &r) == SPT_ERR_INVALID_ARG, "null pcm");
    ip.language = "xx";
    CHECK(spt_transcribe(ctx, pcm, n, &ip, &r) == SPT_ERR_INVALID_ARG, "unknown language");

    spt_timings tm;
    CHECK(spt_get_timings(ctx, &tm) == SPT_OK, "timings");
    spt_ctx_destroy(ctx);
    return 0;
}

/* HipFrameResampler (rust/spittle-hip): create 48 kHz -> 16 kHz with 30 ms frames, one stream,
 * destroy; the output length rule of FrameResampler::finish (resampler.rs:66-86) */
static int resampler_session(void) {
    spt_resampler* r = NULL;
    char err[256] = {0};
    CHECK(spt_resampler_create(48000, 16000, 480, 0, &r, err, sizeof err) == SPT_OK && r, err);
    int32_t nin = 0, nout = 0;
    CHECK(spt_resampler_info(r, &nin, &nout) == SPT_OK && nin == 1026 && nout == 342, "rubato unit sizes");
    const size_t n = 48000 * 2 + 100;
    float* x = (float*)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; ++i) x[i] = 0.5f * sinf(2.0f * 3.14159265f * 1000.0f * (float)i / 48000.0f);
    const size_t need = spt_resample_output_len(r, n);
    /* ceil(n / 1024) chunks of 1024 -> floor(. / 1026) units of 342 -> whole 480-sample frames */
    const size_t units = ((n + 1023) / 1024 * 1024) / 1026;
    CHECK(need == (units * 342 + 479) / 480 * 480, "output length");
    float* y = (float*)malloc(need * sizeof(float));
    size_t got = 0;
    CHECK(spt_resample(r, x, n, y, need - 1, &got) == SPT_ERR_INVALID_ARG, "short output buffer");
    CHECK(spt_resample(r, x, n, y, need, &got) == SPT_OK && got == need, spt_resampler_last_error(r));
    double e = 0.0;
    for (size_t i = 8000; i < 24000; ++i) e += (double)y[i] * y[i];
    CHECK(fabs(sqrt(e / 16000.0) - 0.5 / sqrt(2.0)) < 2e-3, "1 kHz tone keeps its amplitude");
    free(x);
    free(y);
    spt_resampler_destroy(r);
    CHECK(spt_resampler_create(10, 16000, 480, 0, &r, err, sizeof err) == SPT_ERR_INVALID_ARG && !r, "bad rate");
    return 0;
}

/* HipParakeetEngine: load the model directory, transcribe with Segment timestamps, read, free */
static int parakeet_session(const char* dir, const float* pcm, size_t n) {
    spt_pk_model_params mp;
    spt_parakeet_default_model_params(&mp); /* ParakeetModelParams::int8(): fp16 encoder */
    mp.max_batch = 2;
    mp.max_seconds = 8.0f;
    spt_pk_ctx* ctx = NULL;
    char err[512] = {0};
    spt_status st = spt_parakeet_create(dir, &mp, &ctx, err, sizeof err);
    if (st != SPT_OK) fprintf(stderr, "parakeet create: %s\n", err);
    CHECK(st == SPT_OK && ctx, "spt_parakeet_create(model directory)");
    spt_pk_infer_params ip;
    spt_parakeet_default_infer_params(&ip);
    CHECK(ip.timestamp_granularity == SPT_PK_TS_SEGMENT, "Segment granularity by default");
    spt_pk_result* r = NULL;
    st = spt_parakeet_transcribe(ctx, pcm, n, &ip, &r);
    if (st != SPT_OK) fprintf(stderr, "parakeet transcribe: %s\n", spt_parakeet_last_error(ctx));
    CHECK(st == SPT_OK && r && r->text, "spt_parakeet_transcribe");
    for (int i = 0; i < r->n_segments; ++i) CHECK(r->segments[i].end > r->segments[i].start, "segment times");
    printf("parakeet: %d tokens, %d segments, text \"%.60s\"\n", r->n_tokens, r->n_segments, r->text);
    spt_parakeet_result_free(r);
    spt_parakeet_destroy(ctx);
    return 0;
}

/* HipSmoothedVad (rust/spittle-hip): SileroVad::new(path, 0.3) + SmoothedVad::new(.., 15, 15, 2),
 * push_frame per 30 ms frame, reset, destroy (audio.rs:132-134, recorder.rs:284-301) */
static int vad_session(const char* model_path) {
    spt_vad_params p;
    spt_vad_default_params(&p);
    CHECK(p.threshold == 0.3f && p.prefill_frames == 15 && p.hangover_frames == 15 && p.onset_frames == 2,
          "SmoothedVad defaults of the app");
    spt_vad* v = NULL;
    char err[256] = {0};
    spt_status st = spt_vad_create(model_path, &p, &v, err, sizeof err);
    if (st != SPT_OK) fprintf(stderr, "vad create: %s\n", err);
    CHECK(st == SPT_OK && v, "spt_vad_create");
    float frame[480];
    size_t kept = 0;
    int speech = 0;
    for (int f = 0; f < 100; ++f) { /* 3 s: 1 s silence, 1 s voiced tone bursts, 1 s silence */
        for (int i = 0; i < 480; ++i) {
            const float t = (float)(f * 480 + i) / 16000.0f;
            const int voiced = f >= 33 && f < 66;
            frame[i] = voiced ? 0.3f * sinf(2.0f * 3.14159265f * 180.0f * t) * (0.6f + 0.4f * sinf(2.0f * 3.14159265f * 4.0f * t))
                              : 0.0f;
        }
        spt_vad_result* r = NULL;
        CHECK(spt_vad_push(v, frame, 480, &r) == SPT_OK && r, spt_vad_last_error(v));
        CHECK(r->n_frames == 1 && r->prob[0] >= 0.0f && r->prob[0] <= 1.0f, "one frame, a probability");
        CHECK(r->n_samples == 0 || r->n_samples % 480 == 0, "whole frames kept");
        kept += r->n_samples;
        speech += r->kind[0] != 0;
        spt_vad_result_free(r);
    }
    printf("vad: %d speech frames, %zu samples kept\n", speech, kept);
    CHECK(spt_vad_reset(v, 0) == SPT_OK, "reset");
    spt_vad_destroy(v);
    CHECK(spt_vad_create("/nonexistent/silero_vad_v4.onnx", &p, &v, err, sizeof err) != SPT_OK && !v, "missing model");
    return 0;
}

int main(int argc, char** argv) {
    const char* spec = argc > 1 ? argv[1] : "synthetic:tiny";
    printf("%s\n", spt_version());
    spt_ctx* ctx = NULL;
    char err[256];
    CHECK(spt_ctx_create("/nonexistent/ggml-base.bin", NULL, &ctx, err, sizeof err) == SPT_ERR_LOAD && !ctx,
          "missing model file");
    if (argc > 2 && strcmp(argv[2], "--link-only") == 0) {
        if (argc > 3) { /* the model-directory loader needs no device */
            spt_pk_onnx* h = NULL;
            spt_pk_model_info info;
            spt_status st = spt_parakeet_onnx_open(argv[3], &h, &info, err, sizeof err);
            if (st != SPT_OK) fprintf(stderr, "onnx open: %s\n", err);
            CHECK(st == SPT_OK && h, "spt_parakeet_onnx_open");
            printf("parakeet dir: d %d, layers %d, heads %d, vocab %d, %d dequantised\n", info.d, info.n_layers,
                   info.n_heads, info.n_vocab, info.reserved0);
            spt_parakeet_onnx_close(h);
        }
        return 0;
    }
    const size_t n = 16000 * 6;
    float* pcm = (float*)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; ++i)
        pcm[i] = 0.3f * sinf(2.0f * 3.14159265f * 440.0f * (float)i / 16000.0f) +
                 0.05f * sinf(2.0f * 3.14159265f * 1234.5f * (float)i / 16000.0f);
    int rc = one_session(spec, pcm, n);
    if (!rc) rc = one_session(spec, pcm, n); /* unload, then load again */
    if (!rc) rc = resampler_session();
    if (!rc && argc > 3) rc = parakeet_session(argv[3], pcm, n);
    if (!rc && argc > 4) rc = vad_session(argv[4]);
    free(pcm);
    if (!rc) printf("capi_smoke ok\n");
    return rc;
}
