// ubench.cpp -- kernel microbenchmarks (developer tool, not part of the C ABI).
// Times the library's launchers with HIP events, back-to-back launches on one stream.
//   ubench gemv  N K R mode ln dtype [ksplit npend]  mode: 0 bias 1 gelu 2 partial 3 qkv 4 logits 5 resid
//   ubench attn  B H ctx nkeys Tq dtype   self-attention
//   ubench xattn B T splits dtype        cross-attention, 8 layers back to back
//   ubench gemm  M N K epi dtype         128 vs 256 tile (time, bitwise diff)
//   ubench layer B dtype [xsplit]        one large-v3 decoder layer (8 launches)
//   ubench layer2 B dtype [...]          two such chains on two streams
//   ubench null
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
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

// which XCD each block of a launch ran on (HW_REG_XCC_ID)
__global__ void xcc_kernel(int* out) {
    if (threadIdx.x == 0) {
        unsigned v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        out[blockIdx.x] = (int)(v & 0xf);
    }
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
    if (what == "xcc") {
        // block -> XCD placement over a sequence of dependent launches (graph and eager): is block b
        // of every launch on XCD (x0 + b) % 8, and does x0 stay put from one launch to the next?
        const int grids[] = {80, 240, 80, 80, 160, 160, 811, 64, 1, 80, 240, 160};
        const int NG = sizeof(grids) / sizeof(int), REP = 4;
        int* out = (int*)dalloc((size_t)NG * REP * 1024 * 4);
        for (int mode = 0; mode < 2; ++mode) {
            auto run = [&] {
                for (int r = 0; r < REP; ++r)
                    for (int i = 0; i < NG; ++i)
                        hipLaunchKernelGGL(xcc_kernel, dim3(grids[i]), dim3(256), 0, st, out + (size_t)(r * NG + i) * 1024);
            };
            if (mode == 0) {
                hipGraph_t gr;
                hipGraphExec_t ge;
                HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
                run();
                HIP_CHECK(hipStreamEndCapture(st, &gr));
                HIP_CHECK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
                for (int k = 0; k < 3; ++k) HIP_CHECK(hipGraphLaunch(ge, st));
            } else {
                run();
            }
            HIP_CHECK(hipStreamSynchronize(st));
            std::vector<int> h((size_t)NG * REP * 1024);
            HIP_CHECK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
            printf("xcc %s:", mode == 0 ? "graph" : "eager");
            for (int l = 0; l < NG * REP; ++l) {
                const int* o = h.data() + (size_t)l * 1024;
                bool rr = true;
                for (int b = 0; b < grids[l % NG]; ++b) rr = rr && o[b] == (o[0] + b) % 8;
                printf(" %d:%d%s", grids[l % NG], o[0], rr ? "" : "!");
            }
            printf("\n");
        }
        return 0;
    }
    if (what == "chain") {
        // a captured graph of NL dependent launches of one decoder GEMV shape, every launch on its
        // own weights (cache-cold: a 512 MB read precedes each replay), as in the decode loop.
        // kind: 0 null kernel; 1 self/cross-out (resid, A_DIRECT, N=K=1280); 2 cross-Q (LN, N=K=1280);
        // 3 QKV (LN + 2 pending slabs, N=3840); 4 fc1 (LN, GELU, N=5120); 5 fc2 (K=5120, 2 slabs)
        // SPT_STAMP builds print the workgroup timeline: per launch the start of its first workgroup
        // after the previous launch's last end (gap), start spread, first / last end.
        const int kind = ai(2, 1), NL = ai(3, 48), G = ai(4, 80), dt = DT_BF16, d = 1280, B = 8;
        gemv_prepare(dt);
        const int N = kind == 3 ? 3 * d : kind == 4 ? 4 * d : d, K = kind == 5 ? 4 * d : d;
        std::vector<void*> Ws(NL);
        for (int l = 0; l < NL; ++l) Ws[l] = drand((size_t)N * K, dt, 100 + l, -5);
        float* bias = frand(N, 2, -5);
        float* lnw = frand(K, 3, -3);
        float* lnb = frand(K, 4, -4);
        float* x = frand((size_t)B * K, 5, 0);
        void* A = drand((size_t)B * K, dt, 6, 0);
        float* pend = frand((size_t)4 * B * d, 7, -3);
        float* x2 = (float*)dalloc((size_t)B * d * 4);
        void* C = dalloc((size_t)4 * B * N * 4 + 64);
        void* cache = dalloc((size_t)2 * B * 20 * 448 * 64 * 2);
        void* flush = dalloc((size_t)512 << 20);
        unsigned* scratch = (unsigned*)dalloc(64);
        const int maxwg = 1024;
        unsigned long long* stamps = (unsigned long long*)dalloc((size_t)NL * maxwg * 2 * 8);
        int* np = (int*)dalloc(4);
        auto launch = [&](int l) {
            unsigned long long* sp = stamps + (size_t)l * maxwg * 2;
            if (kind == 0) {
                hipLaunchKernelGGL(null_kernel, dim3(G), dim3(512), 0, st, np);
                return;
            }
            GemvArgs a{};
            a.R = B; a.K = K; a.N = N; a.W = Ws[l]; a.bias = bias; a.stamp = sp;
            for (int p = 0; p < kMaxPend; ++p) a.pend[p] = pend + (size_t)p * B * d;
            if (kind == 1) {
                a.A = A; a.lda = K; a.C = x; a.ldc = d;
                gemv(dt, GV_BIAS_RESID, A_DIRECT, a, st);
            } else if (kind == 5) {
                a.A = A; a.lda = K; a.C = pend; a.ldc = d; a.c_split = (int64_t)B * d; a.ksplit = 2;
                a.A = C; a.lda = K;  // any bf16 rows of width K (contents irrelevant)
                gemv(dt, GV_PARTIAL, A_DIRECT, a, st);
            } else {
                a.A = x; a.lda = K; a.ln_w = lnw; a.ln_b = lnb;
                a.n_pend = kind == 3 ? 2 : 0;
                a.x_out = kind == 3 ? x2 : nullptr;
                a.C = C; a.ldc = kind == 3 ? d : N;
                if (kind == 3) {
                    a.cache = cache; a.cache_B = B; a.cache_H = 20; a.cache_ctx = 448; a.Tq = 1; a.st = ds;
                    gemv(dt, GV_QKV_CACHE, A_LN, a, st);
                } else {
                    gemv(dt, kind == 4 ? GV_BIAS_GELU : GV_BIAS, A_LN, a, st);
                }
            }
        };
        HIP_CHECK(hipDeviceSynchronize());
        hipGraph_t g;
        HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int l = 0; l < NL; ++l) launch(l);
        HIP_CHECK(hipStreamEndCapture(st, &g));
        hipGraphExec_t ge;
        HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        double tot = 0;
        const int reps = 6;
        for (int r = 0; r < reps; ++r) {
            cache_flush(flush, (int64_t)512 << 20, scratch, st);
            HIP_CHECK(hipEventRecord(e0, st));
            HIP_CHECK(hipGraphLaunch(ge, st));
            HIP_CHECK(hipEventRecord(e1, st));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) tot += ms;
        }
        const double us = tot * 1000.0 / ((reps - 1) * NL);
        printf("chain kind=%d N=%d K=%d launches=%d : %.2f us per launch  %.0f GB/s\n", kind, N, K, NL, us,
               kind ? (double)N * K * 2 / us / 1e3 : 0.0);
        if (kind > 0) {
            std::vector<unsigned long long> h((size_t)NL * maxwg * 2);
            HIP_CHECK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
            const int nwg = kind == 5 ? 2 * (N / 16) : (kind == 4 ? N / 32 : N / 16);
            double sg = 0, ss = 0, sf = 0, sl = 0;
            unsigned long long prev_end = 0;
            int cnt = 0;
            for (int l = 0; l < NL; ++l) {
                unsigned long long s0 = ~0ull, s1 = 0, e0_ = ~0ull, e1_ = 0;
                for (int w = 0; w < nwg; ++w) {
                    const unsigned long long a0 = h[((size_t)l * maxwg + w) * 2], a1 = h[((size_t)l * maxwg + w) * 2 + 1];
                    s0 = std::min(s0, a0); s1 = std::max(s1, a0); e0_ = std::min(e0_, a1); e1_ = std::max(e1_, a1);
                }
                if (l > 0 && s0 >= prev_end) {
                    sg += (s0 - prev_end) * 0.01; ss += (s1 - s0) * 0.01; sf += (e0_ - s0) * 0.01; sl += (e1_ - s0) * 0.01;
                    ++cnt;
                }
                prev_end = e1_;
            }
            if (cnt)
                printf("  timeline (us, mean over %d launches): gap prev-last-end -> first-start %.2f | start spread %.2f | "
                       "first end %.2f | last end %.2f\n", cnt, sg / cnt, ss / cnt, sf / cnt, sl / cnt);
        }
        return 0;
    }
    if (what == "stream") {  // bandwidth ceiling of a plain coalesced read of NL x 61.4 MB (one per launch)
        const int G = ai(2, 1024), TPB = ai(3, 256), NL = 8;
        const size_t bytes = (size_t)61440000;
        void* buf = dalloc(bytes * NL);
        unsigned* sink = (unsigned*)dalloc(64);
        HIP_CHECK(hipDeviceSynchronize());
        const double us = time_us(st, 10, [&] {
            for (int l = 0; l < NL; ++l) stream_read((const char*)buf + bytes * l, (int64_t)bytes, sink, G, TPB, st);
        }) / NL;
        printf("stream grid=%d x %d : %.2f us per 61.4 MB  %.0f GB/s\n", G, TPB, us, bytes / us / 1e3);
        return 0;
    }
    if (what == "gemv") {
        const int N = ai(2, 1280), K = ai(3, 1280), R = ai(4, 8), mode = ai(5, 2), ln = ai(6, 0), dt = ai(7, DT_BF16),
                  ksplit = ai(8, 1), npend = ai(9, 0);
        gemv_prepare(dt);
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* W = drand((size_t)N * K, dt, 1, -5);
        float* bias = frand(N, 2, -5);
        float* lnw = frand(K, 3, -3);
        float* lnb = frand(K, 4, -4);
        void* A = ln ? (void*)frand((size_t)R * K, 5, 0) : drand((size_t)R * K, dt, 5, 0);
        float* zero = (float*)dalloc((size_t)4 * R * K * 4);
        void* C = dalloc((size_t)4 * R * N * 4 + 64);
        void* cache = dalloc((size_t)2 * R * 20 * 448 * 64 * esz);
        uint32_t* sup = (uint32_t*)dalloc(N / 8 + 64);
        void* part = dalloc((size_t)R * ((N + 15) / 16) * 16 + 64);
        GemvArgs a{};
        a.A = A; a.lda = K; a.R = R; a.W = W; a.N = N; a.K = K; a.bias = bias; a.C = C; a.ldc = N;
        if (ln) { a.ln_w = lnw; a.ln_b = lnb; }
        for (int p = 0; p < kMaxPend; ++p) a.pend[p] = zero + (size_t)p * R * K;
        a.n_pend = npend;
        a.cache = cache; a.cache_B = R; a.cache_H = N / 3 / 64; a.cache_ctx = 448; a.Tq = 1; a.st = ds;
        a.suppress = sup; a.blank0 = a.blank1 = -1; a.part = part; a.n_tiles = (N + 15) / 16;
        a.ksplit = ksplit; a.c_split = (int64_t)R * N;
        if (mode == GV_QKV_CACHE) a.ldc = N / 3;
        const double us = time_us(st, iters, [&] { gemv(dt, mode, ln ? A_LN : A_DIRECT, a, st); });
        const double bytes = (double)N * K * esz;
        printf("gemv N=%d K=%d R=%d mode=%d ln=%d dt=%d ksplit=%d npend=%d : %.2f us  %.0f GB/s\n", N, K, R, mode, ln, dt,
               ksplit, npend, us, bytes / us / 1e3);
        return 0;
    }
    if (what == "attn") {  // self-attention (causal) over nkeys cached keys
        const int B = ai(2, 8), H = ai(3, 20), ctx = ai(4, 448), nk = ai(5, 132), Tq = ai(6, 1), dt = ai(7, DT_BF16);
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* q = drand((size_t)B * Tq * H * 64, dt, 1, 0);
        void* kv = drand((size_t)2 * B * H * ctx * 64, dt, 2, 0);
        void* out = dalloc((size_t)B * Tq * H * 64 * esz);
        DecState h{nk - Tq, 0};
        HIP_CHECK(hipMemcpy(ds, &h, sizeof(h), hipMemcpyHostToDevice));
        const double us = time_us(st, iters, [&] { dec_self_attn(dt, q, kv, B, H, ctx, Tq, ds, out, st); });
        printf("self-attn B=%d H=%d nk=%d Tq=%d dt=%d : %.2f us  %.0f GB/s\n", B, H, nk, Tq, dt, us,
               2.0 * B * H * nk * 64 * esz / us / 1e3);
        return 0;
    }
    if (what == "xattn") {  // cross-attention over T encoder keys of NL layers back to back (cache-cold)
        const int B = ai(2, 8), T = ai(3, 1500), S = ai(4, 1), dt = ai(5, DT_BF16), NL = 8, d = 1280, H = 20;
        const int esz = dt == DT_BF16 ? 2 : 4;
        void* q = drand((size_t)B * d, dt, 1, 0);
        const size_t layer = (size_t)2 * B * H * ((T + 31) / 32 * 32) * 64;
        void* kv = drand(layer * NL, dt, 2, 0);
        void* out = dalloc((size_t)B * d * esz);
        float* part = (float*)dalloc((size_t)B * H * 32 * 66 * 4);
        HIP_CHECK(hipDeviceSynchronize());
        const double us = time_us(st, 10, [&] {
            // S = 9: the blocked [T/32][B][H][2][32][64] layout, one workgroup per (b, h)
            for (int l = 0; l < NL; ++l) dec_cross_attn(dt, q, (const char*)kv + layer * l * esz, B, B, H, T, 1, out, st, S, part);
        }) / NL;
#if SPT_STAMP
        {   // workgroup timeline of one more (cache-cold) launch
            unsigned long long* sp = (unsigned long long*)dalloc((size_t)B * H * 3 * 8);
            void* flush = dalloc((size_t)512 << 20);
            unsigned* sink = (unsigned*)dalloc(64);
            cache_flush(flush, (int64_t)512 << 20, sink, st);
            set_xattn_stamp(sp);
            dec_cross_attn(dt, q, kv, B, B, H, T, 1, out, st, S, part);
            HIP_CHECK(hipStreamSynchronize(st));
            set_xattn_stamp(nullptr);
            std::vector<unsigned long long> h((size_t)B * H * 3);
            HIP_CHECK(hipMemcpy(h.data(), sp, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < B * H; ++i) t0 = std::min(t0, h[3 * i]);
            std::vector<double> st_, str_, end_;
            for (int i = 0; i < B * H; ++i) {
                st_.push_back((h[3 * i] - t0) * 0.01);
                str_.push_back((h[3 * i + 1] - t0) * 0.01);
                end_.push_back((h[3 * i + 2] - t0) * 0.01);
            }
            auto q5 = [](std::vector<double> v) {
                std::sort(v.begin(), v.end());
                char b[128];
                snprintf(b, sizeof b, "min %.2f med %.2f max %.2f", v.front(), v[v.size() / 2], v.back());
                return std::string(b);
            };
            printf("  timeline us from first start: start %s | wave0 streamed %s | merged %s\n", q5(st_).c_str(),
                   q5(str_).c_str(), q5(end_).c_str());
        }
#endif
        printf("cross-attn B=%d T=%d splits=%d dt=%d (8 layers back to back) : %.2f us  %.0f GB/s\n", B, T, S, dt, us,
               2.0 * B * H * T * 64 * esz / us / 1e3);
        return 0;
    }
    if (what == "gemm") {  // 128 x 128 vs 256 x 256 tile: timing and bitwise agreement
        const int M = ai(2, 12000), N = ai(3, 5120), K = ai(4, 1280), epi = ai(5, 0), dt = ai(6, DT_BF16), ks = ai(7, 1);
        void* A = drand((size_t)M * K, dt, 1, -2);
        void* W = drand((size_t)N * K, dt, 2, -5);
        float* bias = frand(N, 3, -5);
        const size_t cbytes = (size_t)ks * M * N * 4;
        void* C = dalloc(cbytes);
        float* C0 = frand(cbytes / 4, 5, 0);  // the residual operand of EPI_BIAS_RESID (C += alpha * v)
        GemmArgs g{};
        g.alpha = 1.0f;
        g.A = A; g.lda = K; g.W = W; g.ldw = K; g.M = M; g.N = N; g.K = K; g.bias = bias; g.C = C; g.ldc = N;
        g.kv_B = M / 1500; g.kv_T = 1500; g.kv_H = 20; g.ksplit = ks; g.c_split = (int64_t)M * N;
        if (epi == EPI_BIAS_GELU_POS) g.pos = frand((size_t)M * N, 4, 0);
        HIP_CHECK(hipDeviceSynchronize());  // inputs are generated on the null stream
        std::vector<char> ref(cbytes), out(cbytes);
        double us[7] = {0, 0, 0, 0, 0, 0, 0};
        std::vector<char> out64(cbytes), out6464(cbytes), outring(cbytes);
        const bool ring = dt != DT_F32 && N % 64 == 0;
        for (int v : {1, 2, 4, 5, 6}) {
            if (v == 6 && !ring) continue;
            HIP_CHECK(hipMemcpyAsync(C, C0, cbytes, hipMemcpyDeviceToDevice, st));
            gemm_nt_variant(dt, epi, g, 1, v, st);
            HIP_CHECK(hipStreamSynchronize(st));
            HIP_CHECK(hipMemcpy(v == 1 ? ref.data() : v == 2 ? out.data() : v == 4 ? out64.data() : v == 5 ? out6464.data() : outring.data(),
                                C, cbytes, hipMemcpyDeviceToHost));
            us[v] = time_us(st, 20, [&] { gemm_nt_variant(dt, epi, g, 1, v, st); });
        }
        size_t diff64 = 0, diff6464 = 0, diffring = 0;
        for (size_t i = 0; i < cbytes; ++i) {
            diff64 += ref[i] != out64[i];
            diff6464 += ref[i] != out6464[i];
            diffring += ring && ref[i] != outring[i];
        }
        if (ring) printf("ring 208x64: %.2f us %.1f TF/s, bytes differing from 128-tile %zu\n", us[6], 2.0 * M * N * K / us[6] / 1e6, diffring);
        size_t diff = 0, shown = 0;
        for (size_t i = 0; i < cbytes; ++i) {
            if (ref[i] == out[i]) continue;
            ++diff;
            if (shown < 6 && epi == EPI_KVSPLIT && (i & 1) == 0) {  // decode [L][2][B][H][T][64] bf16
                const size_t e = i / 2, el = e % 64, t = e / 64 % 1500, h = e / 64 / 1500 % 20, bb = e / 64 / 1500 / 20 % g.kv_B,
                             lk = e / 64 / 1500 / 20 / g.kv_B;
                const size_t row = bb * 1500 + t, col = (lk / 2) * 2560 + (lk % 2) * 1280 + h * 64 + el;
                printf("  diff at row %zu col %zu: 128=%04x 256=%04x\n", row, col, ((uint16_t*)ref.data())[e], ((uint16_t*)out.data())[e]);
                ++shown;
            }
        }
        const double fl = 2.0 * M * N * K;
        printf("gemm M=%d N=%d K=%d ks=%d epi=%d dt=%d : 128-tile %.2f us %.1f TF/s | 256-tile %.2f us %.1f TF/s | bytes differing %zu"
               " | 64x128 %.2f us %.1f TF/s, bytes differing from 128-tile %zu | 64x64 %.2f us, differing %zu\n",
               M, N, K, ks, epi, dt, us[1], fl / us[1] / 1e6, us[2], fl / us[2] / 1e6, diff, us[4], fl / us[4] / 1e6, diff64,
               us[5], diff6464);
        return 0;
    }
    if (what == "layer" || what == "layer2") {
        // layer: one large-v3 decoder layer chain at batch B
        // layer2: two independent chains of batch B on two streams (can they overlap?)
        const int B = ai(2, 8), dt = ai(3, DT_BF16), xs = ai(4, 1), d = 1280, H = 20, ctx = 448, T = 1500;
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
        float* zero = (float*)dalloc((size_t)B * d * 4);
        struct Chain { float *x, *x2, *pend, *xpart; void *q, *ao, *ff, *skv, *ckv; DecState* ds; };
        auto mk = [&](uint32_t s) {
            Chain c;
            c.x = frand((size_t)B * d, 10 + s, 0);
            c.x2 = (float*)dalloc((size_t)B * d * 4);
            c.pend = (float*)dalloc((size_t)kMaxPend * B * d * 4);
            c.xpart = (float*)dalloc((size_t)B * H * 4 * 66 * 4);
            c.q = dalloc((size_t)B * d * esz);
            c.ao = dalloc((size_t)B * d * esz);
            c.ff = dalloc((size_t)B * 4 * d * esz);
            c.skv = drand((size_t)2 * B * H * ctx * 64, dt, 11 + s, 0);
            c.ckv = drand((size_t)2 * B * H * T * 64, dt, 12 + s, 0);
            c.ds = (DecState*)dalloc(64);
            DecState h{128, 0};
            HIP_CHECK(hipMemcpy(c.ds, &h, sizeof(h), hipMemcpyHostToDevice));
            return c;
        };
        // the engine's layer (Engine::enqueue_decoder_pass): 8 launches, pending slabs after the
        // self-out (2) and fc2 (4) projections; the chain starts with fc2's 4 slabs pending
        const int fs = getenv("FC2S") ? atoi(getenv("FC2S")) : 2;  // fc2 K split (pending slabs)
        const int sos = getenv("SOS") ? atoi(getenv("SOS")) : 2;   // self-out K split
        auto layer = [&](const Chain& c, hipStream_t s) {
            float *xc = c.x, *xo = c.x2;
            int np = fs > 1 ? fs : 0;
            auto ln_input = [&](GemvArgs& a) {
                a.A = xc;
                for (int p = 0; p < kMaxPend; ++p) a.pend[p] = p < np ? c.pend + (size_t)p * B * d : zero;
                a.n_pend = np;
                a.x_out = np ? xo : nullptr;
            };
            auto consumed = [&] { if (np > 0) std::swap(xc, xo); np = 0; };
            GemvArgs a{};
            ln_input(a); a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B;
            a.W = wqkv; a.N = 3 * d; a.K = d; a.bias = b4;
            a.C = c.q; a.ldc = d; a.cache = c.skv; a.cache_B = B; a.cache_H = H; a.cache_ctx = ctx; a.Tq = 1; a.st = c.ds;
            gemv(dt, GV_QKV_CACHE, A_LN, a, s);
            consumed();
            dec_self_attn(dt, c.q, c.skv, B, H, ctx, 1, c.ds, c.ao, s);
            a = GemvArgs{};
            a.A = c.ao; a.lda = d; a.R = B; a.W = wo; a.N = d; a.K = d; a.bias = b4;
            if (sos > 1) {
                a.C = c.pend; a.ldc = d; a.c_split = (int64_t)B * d; a.ksplit = sos; np = sos;
                gemv(dt, GV_PARTIAL, A_DIRECT, a, s);
            } else {  // straight into the residual
                a.C = xc; a.ldc = d;
                gemv(dt, GV_BIAS_RESID, A_DIRECT, a, s);
            }
            a = GemvArgs{};
            ln_input(a); a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B;
            a.W = wq; a.N = d; a.K = d; a.bias = b4; a.C = c.q; a.ldc = d;
            gemv(dt, GV_BIAS, A_LN, a, s);
            consumed();
            dec_cross_attn(dt, c.q, c.ckv, B, B, H, T, 1, c.ao, s, xs, c.xpart);
            a = GemvArgs{};
            a.A = c.ao; a.lda = d; a.R = B; a.W = wco; a.N = d; a.K = d; a.bias = b4; a.C = xc; a.ldc = d;
            if (xs > 1) { a.apart = c.xpart; a.a_splits = xs; a.a_heads = H; }
            gemv(dt, GV_BIAS_RESID, xs > 1 ? A_ATTN : A_DIRECT, a, s);
            a = GemvArgs{};
            ln_input(a); a.lda = d; a.ln_w = lnw; a.ln_b = lnb; a.R = B;
            a.W = w1; a.N = 4 * d; a.K = d; a.bias = b4; a.C = c.ff; a.ldc = 4 * d;
            gemv(dt, GV_BIAS_GELU, A_LN, a, s);
            consumed();
            a = GemvArgs{};
            a.A = c.ff; a.lda = 4 * d; a.R = B; a.W = w2; a.N = d; a.K = 4 * d; a.bias = b4;
            if (fs > 1) {
                a.C = c.pend; a.ldc = d; a.c_split = (int64_t)B * d; a.ksplit = fs; np = fs;
                gemv(dt, GV_PARTIAL, A_DIRECT, a, s);
            } else {
                a.C = xc; a.ldc = d;
                gemv(dt, GV_BIAS_RESID, A_DIRECT, a, s);
            }
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
