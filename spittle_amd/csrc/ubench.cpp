// ubench.cpp -- kernel microbenchmarks (developer tool, not part of the C ABI).
// Times the library's launchers with HIP events, back-to-back launches on one stream.
//   ubench gemv  N K R mode ln dtype     mode: 0 bias 1 gelu 2 resid 3 qkv 4 logits
//   ubench attn  B H ctx nkeys causal Tq dtype [splits waves]
//   ubench gemm  M N K epi dtype
//   ubench layer B dtype [xsplits xwaves] one large-v3 decoder layer (8 launches)
//   ubench layer2 B dtype [...]          two such chains on two streams
//   ubench null
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"

using namespace spt;

static void* dalloc(size_t bytes) {
    void* p;
    HIP_CHECK(hipMalloc(&p, bytes));
    HIP_CHECK(hipMemset(p, 0, bytes));
    return p;
}
static void* drand(size_t n, int dt, uint32_t tid, int e) {
    void* p = dalloc(n * (dt == DT_BF16 ? 2 : 4));
    gen_weights(dt, p, (int64_t)n, 7, tid, WK_MAT, e, 0);
    return p;
}
static float* frand(size_t n, uint32_t tid, int e) { return (float*)drand(n, DT_F32, tid, e); }

static double time_us(hipStream_t st, int iters, const std::function<void()>& f) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipEventRecord(a, st));
    for (int i = 0; i < iters; ++i) f();
    HIP_CHECK(hipEventRecord(b, st));
    HIP_CHECK(hipEventSynchronize(b));
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0 / iters;
}

__global__ void null_kernel(int* p) {
    if (threadIdx.x == 1023 && blockIdx.x == 100000) *p = 1;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: ubench gemv|attn|gemm|layer|null ...\n");
        return 2;
    }
    const std::string what = argv[1];
    auto ai = [&](int i, int dflt) { return argc > i ? atoi(argv[i]) : dflt; };
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int iters = 200;
    DecState* ds = (DecState*)dalloc(64);
    if (what == "null") {
        int* p = (int*)dalloc(4);
        for (int g : {1, 80, 256, 1024}) {
            double us = time_us(st, iters, [&] { hipLaunchKernelGGL(null_kernel, dim3(g), dim3(256), 0, st, p); });
            printf("null grid=%d : %.2f us\n", g, us);
        }
        return 0;
    }
    if (what == "gemv") {
        const int N = ai(2, 1280), K = ai(3, 1280), R = ai(4, 8), mode = ai(5, 2), ln = ai(6, 0), dt = ai(7, DT_BF16);
        gemv_prepare(dt);
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* W = drand((size_t)N * K, dt, 1, -5);
        float* bias = frand(N, 2, -5);
        float* lnw = frand(K, 3, -3);
        float* lnb = frand(K, 4, -4);
        void* A = ln ? (void*)frand((size_t)R * K, 5, 0) : drand((size_t)R * K, dt, 5, 0);
        void* C = dalloc((size_t)R * N * 4 + 64);
        void* cache = dalloc((size_t)2 * R * 20 * 448 * 64 * esz);
        uint32_t* sup = (uint32_t*)dalloc(N / 8 + 64);
        void* part = dalloc((size_t)R * ((N + 15) / 16) * 16 + 64);
        GemvArgs a{};
        a.A = A; a.lda = K; a.R = R; a.W = W; a.N = N; a.K = K; a.bias = bias; a.C = C; a.ldc = N;
        if (ln) { a.ln_w = lnw; a.ln_b = lnb; }
        a.cache = cache; a.cache_B = R; a.cache_H = N / 3 / 64; a.cache_ctx = 448; a.Tq = 1; a.st = ds;
        a.suppress = sup; a.blank0 = a.blank1 = -1; a.part = part; a.n_tiles = (N + 15) / 16;
        if (mode == GV_QKV_CACHE) a.ldc = N / 3;
        const double us = time_us(st, iters, [&] { gemv(dt, mode, a, st); });
        const double bytes = (double)N * K * esz;
        printf("gemv N=%d K=%d R=%d mode=%d ln=%d dt=%d : %.2f us  %.0f GB/s\n", N, K, R, mode, ln, dt, us,
               bytes / us / 1e3);
        return 0;
    }
    if (what == "attn") {
        const int B = ai(2, 8), H = ai(3, 20), ctx = ai(4, 1500), nk = ai(5, 1500), causal = ai(6, 0),
                  Tq = ai(7, 1), dt = ai(8, DT_BF16);
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* q = drand((size_t)B * Tq * H * 64, dt, 1, 0);
        void* kv = drand((size_t)2 * B * H * ctx * 64, dt, 2, 0);
        void* out = dalloc((size_t)B * Tq * H * 64 * esz);
        DecState h{nk - Tq, 0};
        HIP_CHECK(hipMemcpy(ds, &h, sizeof(h), hipMemcpyHostToDevice));
        double us;
        if (causal) us = time_us(st, iters, [&] { dec_self_attn(dt, q, kv, B, H, ctx, Tq, ds, out, st); });
        else {
            AttnSplit xs;
            xs.splits = ai(9, 1); xs.waves = ai(10, 8);
            xs.xpart = (float*)dalloc((size_t)B * H * kAttnMaxSplit * 4 * 66 * 4);
            xs.xcnt = (unsigned*)dalloc((size_t)B * H * 4);
            us = time_us(st, iters, [&] { dec_cross_attn(dt, q, kv, B, B, H, ctx, Tq, out, xs, st); });
            printf("  (splits=%d waves=%d) ", xs.splits, xs.waves);
        }
        const double bytes = 2.0 * B * H * nk * 64 * esz;
        printf("attn B=%d H=%d nk=%d causal=%d Tq=%d dt=%d : %.2f us  %.0f GB/s\n", B, H, nk, causal, Tq, dt, us,
               bytes / us / 1e3);
        return 0;
    }
    if (what == "gemm") {
        const int M = ai(2, 12000), N = ai(3, 5120), K = ai(4, 1280), epi = ai(5, 0), dt = ai(6, DT_BF16);
        void* A = drand((size_t)M * K, dt, 1, -2);
        void* W = drand((size_t)N * K, dt, 2, -5);
        float* bias = frand(N, 3, -5);
        void* C = dalloc((size_t)M * N * 4);
        GemmArgs g{};
        g.A = A; g.lda = K; g.W = W; g.ldw = K; g.M = M; g.N = N; g.K = K; g.bias = bias; g.C = C; g.ldc = N;
        g.kv_B = M / 1500; g.kv_T = 1500; g.kv_H = 20;
        const double us = time_us(st, 20, [&] { gemm_nt(dt, epi, g, 1, st); });
        printf("gemm M=%d N=%d K=%d epi=%d dt=%d : %.2f us  %.1f TFLOP/s\n", M, N, K, epi, dt, us,
               2.0 * M * N * K / us / 1e6);
        return 0;
    }
    if (what == "layer" || what == "layer2") {
        // layer: one large-v3 decoder layer chain at batch B
        // layer2: two independent chains of batch B on two streams (can they overlap?)
        const int B = ai(2, 8), dt = ai(3, DT_BF16), d = 1280, H = 20, ctx = 448, T = 1500;
        const int xsplits = ai(4, 1), xwaves = ai(5, 8);
        gemv_prepare(dt);
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* wqkv = drand((size_t)3 * d * d, dt, 1, -4);
        void* wo = drand((size_t)d * d, dt, 2, -4);
        void* wq = drand((size_t)d * d, dt, 3, -4);
        void* wco = drand((size_t)d * d, dt, 4, -4);
        void* w1 = drand((size_t)4 * d * d, dt, 5, -4);
        void* w2 = drand((size_t)4 * d * d, dt, 6, -5);
        float* b4 = frand(4 * d, 7, -5);
        float* lnw = frand(d, 8, -3);
        float* lnb = frand(d, 9, -4);
        struct Chain { float* x; void *q, *ao, *ff, *skv, *ckv; DecState* ds; AttnSplit xs; };
        auto mk = [&](uint32_t s) {
            Chain c;
            c.x = frand((size_t)B * d, 10 + s, 0);
            c.q = dalloc((size_t)B * d * esz);
            c.ao = dalloc((size_t)B * d * esz);
            c.ff = dalloc((size_t)B * 4 * d * esz);
            c.skv = drand((size_t)2 * B * H * ctx * 64, dt, 11 + s, 0);
            c.ckv = drand((size_t)2 * B * H * T * 64, dt, 12 + s, 0);
            c.ds = (DecState*)dalloc(64);
            c.xs.splits = xsplits; c.xs.waves = xwaves;
            c.xs.xpart = (float*)dalloc((size_t)B * H * kAttnMaxSplit * 4 * 66 * 4);
            c.xs.xcnt = (unsigned*)dalloc((size_t)B * H * 4);
            DecState h{128, 0};
            HIP_CHECK(hipMemcpy(c.ds, &h, sizeof(h), hipMemcpyHostToDevice));
            return c;
        };
        auto layer = [&](const Chain& c, hipStream_t s) {
            GemvArgs a{};
            a.A = c.x; a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B; a.W = wqkv; a.N = 3 * d; a.K = d; a.bias = b4;
            a.C = c.q; a.ldc = d; a.cache = c.skv; a.cache_B = B; a.cache_H = H; a.cache_ctx = ctx; a.Tq = 1; a.st = c.ds;
            gemv(dt, GV_QKV_CACHE, a, s);
            dec_self_attn(dt, c.q, c.skv, B, H, ctx, 1, c.ds, c.ao, s);
            a = GemvArgs{};
            a.A = c.ao; a.lda = d; a.R = B; a.W = wo; a.N = d; a.K = d; a.bias = b4; a.C = c.x; a.ldc = d;
            gemv(dt, GV_BIAS_RESID, a, s);
            a = GemvArgs{};
            a.A = c.x; a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B; a.W = wq; a.N = d; a.K = d; a.bias = b4;
            a.C = c.q; a.ldc = d;
            gemv(dt, GV_BIAS, a, s);
            dec_cross_attn(dt, c.q, c.ckv, B, B, H, T, 1, c.ao, c.xs, s);
            a = GemvArgs{};
            a.A = c.ao; a.lda = d; a.R = B; a.W = wco; a.N = d; a.K = d; a.bias = b4; a.C = c.x; a.ldc = d;
            gemv(dt, GV_BIAS_RESID, a, s);
            a = GemvArgs{};
            a.A = c.x; a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B; a.W = w1; a.N = 4 * d; a.K = d; a.bias = b4;
            a.C = c.ff; a.ldc = 4 * d;
            gemv(dt, GV_BIAS_GELU, a, s);
            a = GemvArgs{};
            a.A = c.ff; a.lda = 4 * d; a.R = B; a.W = w2; a.N = d; a.K = 4 * d; a.bias = b4; a.C = c.x; a.ldc = d;
            gemv(dt, GV_BIAS_RESID, a, s);
        };
        const double bytes = (14.0 * d * d) * esz + 2.0 * B * H * (T + 129) * 64 * esz;
        Chain c0 = mk(0);
        if (what == "layer") {
            const double eager = time_us(st, 50, [&] { layer(c0, st); });
            hipGraph_t g;
            HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < 8; ++i) layer(c0, st);
            HIP_CHECK(hipStreamEndCapture(st, &g));
            hipGraphExec_t ge;
            HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            const double graph = time_us(st, 20, [&] { HIP_CHECK(hipGraphLaunch(ge, st)); }) / 8;
            printf("layer B=%d dt=%d : eager %.2f us  graph %.2f us  (%.0f GB/s at graph)\n", B, dt, eager, graph,
                   bytes / graph / 1e3);
            return 0;
        }
        Chain c1 = mk(100);
        hipStream_t s2;
        HIP_CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        hipEvent_t fork, join;
        HIP_CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
        // sequential: both chains on one stream; concurrent: second chain on s2
        const double seq = time_us(st, 50, [&] { layer(c0, st); layer(c1, st); });
        const double conc = time_us(st, 50, [&] {
            HIP_CHECK(hipEventRecord(fork, st));
            HIP_CHECK(hipStreamWaitEvent(s2, fork, 0));
            layer(c0, st);
            layer(c1, s2);
            HIP_CHECK(hipEventRecord(join, s2));
            HIP_CHECK(hipStreamWaitEvent(st, join, 0));
        });
        // graphs: one graph per stream, 8 layers each, launched on both streams at once
        hipGraphExec_t ge[2];
        hipStream_t ss[2] = {st, s2};
        Chain* cc[2] = {&c0, &c1};
        for (int k = 0; k < 2; ++k) {
            hipGraph_t g;
            HIP_CHECK(hipStreamBeginCapture(ss[k], hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < 8; ++i) layer(*cc[k], ss[k]);
            HIP_CHECK(hipStreamEndCapture(ss[k], &g));
            HIP_CHECK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
        }
        const double gconc = time_us(st, 20, [&] {
            HIP_CHECK(hipEventRecord(fork, st));
            HIP_CHECK(hipStreamWaitEvent(s2, fork, 0));
            HIP_CHECK(hipGraphLaunch(ge[0], st));
            HIP_CHECK(hipGraphLaunch(ge[1], s2));
            HIP_CHECK(hipEventRecord(join, s2));
            HIP_CHECK(hipStreamWaitEvent(st, join, 0));
        }) / 8;
        printf("layer2 B=%d x2 dt=%d : sequential %.2f us  two-stream eager %.2f us  two-stream graphs %.2f us (per layer pair)\n",
               B, dt, seq, conc, gconc);
        return 0;
    }
    fprintf(stderr, "unknown bench %s\n", what.c_str());
    return 2;
}
