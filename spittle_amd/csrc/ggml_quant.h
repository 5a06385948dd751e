// ggml_quant.h -- ggml's block formats, dequantised by one routine shared by the host
// (ggml_file.cpp: conv kernels, the test hook) and the device (k_init.hip: every matrix).
//
// Restated from ggml-quants.h / ggml-quants.c (dequantize_row_*), the ggml that whisper-rs-sys
// 0.11.1 vendors (/root/reference/src-tauri/Cargo.lock:8156-8174; not vendored here):
//   q4_0  {f16 d; u8 qs[16]}              x = (q - 8) d
//   q4_1  {f16 d, m; u8 qs[16]}           x = q d + m
//   q5_0  {f16 d; u32 qh; u8 qs[16]}      x = (q - 16) d        (bit 4 of element j: qh bit j)
//   q5_1  {f16 d, m; u32 qh; u8 qs[16]}   x = q d + m
//   q8_0  {f16 d; i8 qs[32]}              x = q d
//   (32-element blocks; element j < 16 in the low nibble of qs[j], j + 16 in the high one)
//   q4_K  {f16 d, dmin; u8 scales[12]; u8 qs[128]}           256 = 8 sub-blocks of 32 with
//   q5_K  {f16 d, dmin; u8 scales[12]; u8 qh[32]; u8 qs[128]}  6-bit scale / min codes:
//         x = (d sc) q - (dmin m)
//   q6_K  {u8 ql[128]; u8 qh[64]; i8 scales[16]; f16 d}      x = (d sc) (q - 32)
// Products and sums are rounded one at a time (no fused multiply-add) on both sides.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace spt {

enum { GQ_F32 = 0, GQ_F16 = 1, GQ_Q4_0 = 2, GQ_Q4_1 = 3, GQ_Q5_0 = 6, GQ_Q5_1 = 7, GQ_Q8_0 = 8,
       GQ_Q4_K = 12, GQ_Q5_K = 13, GQ_Q6_K = 14 };

// elements and bytes per block; 0 / 0 for an unsupported type
__host__ __device__ inline void ggml_block_geom(int type, int* blck, int* bytes) {
    switch (type) {
        case GQ_F32: *blck = 1; *bytes = 4; return;
        case GQ_F16: *blck = 1; *bytes = 2; return;
        case GQ_Q4_0: *blck = 32; *bytes = 18; return;
        case GQ_Q4_1: *blck = 32; *bytes = 20; return;
        case GQ_Q5_0: *blck = 32; *bytes = 22; return;
        case GQ_Q5_1: *blck = 32; *bytes = 24; return;
        case GQ_Q8_0: *blck = 32; *bytes = 34; return;
        case GQ_Q4_K: *blck = 256; *bytes = 144; return;
        case GQ_Q5_K: *blck = 256; *bytes = 176; return;
        case GQ_Q6_K: *blck = 256; *bytes = 210; return;
        default: *blck = 0; *bytes = 0; return;
    }
}

__host__ __device__ inline float gq_half(const uint8_t* p) {
    const uint16_t h = (uint16_t)p[0] | ((uint16_t)p[1] << 8);
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, u;
    if (e == 0) {
        if (m == 0) u = s;
        else {  // subnormal: normalise
            e = 127 - 15 + 1;
            while (!(m & 0x400u)) { m <<= 1; --e; }
            u = s | (e << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        u = s | 0x7f800000u | (m << 13);
    } else {
        u = s | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// 6-bit scale and min codes of sub-block j of a q4_K / q5_K block (ggml get_scale_min_k4)
__host__ __device__ inline void gq_scale_min_k4(int j, const uint8_t* q, int* sc, int* mn) {
    if (j < 4) {
        *sc = q[j] & 63;
        *mn = q[j + 4] & 63;
    } else {
        *sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *mn = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

// dequantise one block (blck elements) of a quantised type: out(i, value) for i in [0, blck)
template <typename Out>
__host__ __device__ inline void ggml_dequant_block(int type, const uint8_t* p, Out out) {
#pragma clang fp contract(off)
    switch (type) {
        case GQ_Q8_0: {
            const float d = gq_half(p);
            for (int j = 0; j < 32; ++j) out(j, (float)(int8_t)p[2 + j] * d);
            return;
        }
        case GQ_Q4_0:
        case GQ_Q4_1:
        case GQ_Q5_0:
        case GQ_Q5_1: {
            const bool has_m = type == GQ_Q4_1 || type == GQ_Q5_1, q5 = type == GQ_Q5_0 || type == GQ_Q5_1;
            const float d = gq_half(p), m = has_m ? gq_half(p + 2) : 0.0f;
            const uint8_t* q = p + (has_m ? 4 : 2);
            uint32_t qh = 0;
            if (q5) {
                qh = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
                q += 4;
            }
            const int off = type == GQ_Q4_0 ? 8 : type == GQ_Q5_0 ? 16 : 0;
            for (int j = 0; j < 16; ++j) {
                int x0 = q[j] & 0xf, x1 = q[j] >> 4;
                if (q5) {
                    x0 |= ((qh >> j) << 4) & 0x10;
                    x1 |= (qh >> (j + 12)) & 0x10;
                }
                float v0 = (float)(x0 - off) * d, v1 = (float)(x1 - off) * d;
                if (has_m) {
                    v0 = v0 + m;
                    v1 = v1 + m;
                }
                out(j, v0);
                out(j + 16, v1);
            }
            return;
        }
        case GQ_Q4_K:
        case GQ_Q5_K: {
            const bool q5 = type == GQ_Q5_K;
            const float d = gq_half(p), dmin = gq_half(p + 2);
            const uint8_t* sc = p + 4;
            const uint8_t* qh = p + 16;
            const uint8_t* ql = p + (q5 ? 48 : 16);
            for (int g = 0; g < 4; ++g) {  // 64 elements: sub-blocks 2g (low nibbles), 2g + 1 (high)
                int s0, m0, s1, m1;
                gq_scale_min_k4(2 * g, sc, &s0, &m0);
                gq_scale_min_k4(2 * g + 1, sc, &s1, &m1);
                const float d0 = d * (float)s0, n0 = dmin * (float)m0;
                const float d1 = d * (float)s1, n1 = dmin * (float)m1;
                for (int l = 0; l < 32; ++l) {
                    int a = ql[32 * g + l] & 0xF, b = ql[32 * g + l] >> 4;
                    if (q5) {
                        a += (qh[l] >> (2 * g)) & 1 ? 16 : 0;
                        b += (qh[l] >> (2 * g + 1)) & 1 ? 16 : 0;
                    }
                    out(64 * g + l, d0 * (float)a - n0);
                    out(64 * g + 32 + l, d1 * (float)b - n1);
                }
            }
            return;
        }
        case GQ_Q6_K: {
            const uint8_t* ql = p;
            const uint8_t* qh = p + 128;
            const int8_t* sc = (const int8_t*)(p + 192);
            const float d = gq_half(p + 208);
            for (int h = 0; h < 2; ++h)  // two halves of 128
                for (int l = 0; l < 32; ++l) {
                    const int is = l / 16;
                    const uint8_t a = ql[64 * h + l], b = ql[64 * h + l + 32], c = qh[32 * h + l];
                    const int q1 = ((a & 0xF) | (((c >> 0) & 3) << 4)) - 32;
                    const int q2 = ((b & 0xF) | (((c >> 2) & 3) << 4)) - 32;
                    const int q3 = ((a >> 4) | (((c >> 4) & 3) << 4)) - 32;
                    const int q4 = ((b >> 4) | (((c >> 6) & 3) << 4)) - 32;
                    const int8_t* s = sc + 8 * h;
                    out(128 * h + l, d * (float)s[is + 0] * (float)q1);
                    out(128 * h + l + 32, d * (float)s[is + 2] * (float)q2);
                    out(128 * h + l + 64, d * (float)s[is + 4] * (float)q3);
                    out(128 * h + l + 96, d * (float)s[is + 6] * (float)q4);
                }
            return;
        }
        default:
            return;
    }
}

}  // namespace spt
