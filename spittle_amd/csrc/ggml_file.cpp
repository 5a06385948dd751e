// ggml_file.cpp -- see ggml_file.h.  Host side of model loading only: the bulk
// dequantisation of the weight matrices runs on the device (k_init.hip ggml_dequant).
#include "ggml_file.h"

#include <fcntl.h>
#include <math.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace spt {

namespace {

float h2f(uint16_t h) {  // IEEE half -> float
    const uint32_t s = (uint32_t)(h & 0x8000) << 16;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t u;
    if (e == 0) {
        if (m == 0) u = s;
        else {  // subnormal
            e = 127 - 15 + 1;
            while (!(m & 0x400)) { m <<= 1; --e; }
            m &= 0x3ff;
            u = s | (e << 23) | (m << 13);
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

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;
    template <typename T> T get() {
        T v{};
        if ((size_t)(end - p) < sizeof(T)) { ok = false; return v; }
        memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    const uint8_t* take(size_t n) {
        if ((size_t)(end - p) < n) { ok = false; return nullptr; }
        const uint8_t* r = p;
        p += n;
        return r;
    }
};

}  // namespace

void GgmlFile::type_block(int type, int* blck, int* bytes) {
    switch (type) {
        case GG_F32: *blck = 1; *bytes = 4; return;
        case GG_F16: *blck = 1; *bytes = 2; return;
        case GG_Q4_0: *blck = 32; *bytes = 18; return;
        case GG_Q4_1: *blck = 32; *bytes = 20; return;
        case GG_Q5_0: *blck = 32; *bytes = 22; return;
        case GG_Q5_1: *blck = 32; *bytes = 24; return;
        case GG_Q8_0: *blck = 32; *bytes = 34; return;
        default: *blck = 0; *bytes = 0; return;
    }
}

GgmlFile::~GgmlFile() {
    if (map_) munmap(map_, size_);
}

bool GgmlFile::open(const std::string& path, std::string* err) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) { *err = "cannot open " + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 4) { ::close(fd); *err = "cannot stat " + path; return false; }
    size_ = (size_t)st.st_size;
    map_ = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (map_ == MAP_FAILED) { map_ = nullptr; *err = "cannot map " + path; return false; }
    Reader r{(const uint8_t*)map_, (const uint8_t*)map_ + size_};
    if (r.get<uint32_t>() != 0x67676d6cu) { *err = "not a ggml whisper model (bad magic)"; return false; }
    int32_t h[11];
    for (int i = 0; i < 11; ++i) h[i] = r.get<int32_t>();
    hp_ = GgmlHparams{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10]};
    n_mel_ = r.get<int32_t>();
    n_fft_ = r.get<int32_t>();
    if (!r.ok || n_mel_ <= 0 || n_mel_ > 512 || n_fft_ <= 0 || n_fft_ > 4096) { *err = "bad mel filter header"; return false; }
    const float* fl = (const float*)r.take((size_t)n_mel_ * n_fft_ * 4);
    if (!fl) { *err = "truncated mel filters"; return false; }
    filters_.assign(fl, fl + (size_t)n_mel_ * n_fft_);
    const int32_t nv = r.get<int32_t>();
    if (!r.ok || nv < 0 || nv > 1000000) { *err = "bad vocabulary size"; return false; }
    vocab_.resize(nv);
    for (int i = 0; i < nv; ++i) {
        const uint32_t len = r.get<uint32_t>();
        const uint8_t* s = r.take(len);
        if (!r.ok) { *err = "truncated vocabulary"; return false; }
        vocab_[i].assign((const char*)s, len);
    }
    while (r.ok && r.p < r.end) {
        GgmlTensor t;
        t.n_dims = r.get<int32_t>();
        const int32_t nlen = r.get<int32_t>();
        t.type = r.get<int32_t>();
        if (!r.ok || t.n_dims < 1 || t.n_dims > 4 || nlen <= 0 || nlen > 256) { *err = "bad tensor header"; return false; }
        for (int i = 0; i < t.n_dims; ++i) {
            t.ne[i] = r.get<int32_t>();
            if (t.ne[i] <= 0) { *err = "bad tensor shape"; return false; }
        }
        const uint8_t* nm = r.take(nlen);
        if (!nm) { *err = "truncated tensor name"; return false; }
        t.name.assign((const char*)nm, nlen);
        int blck, bytes;
        type_block(t.type, &blck, &bytes);
        if (!blck) { *err = "unsupported ggml type " + std::to_string(t.type) + " of " + t.name; return false; }
        if (t.ne[0] % blck) { *err = "row length not a multiple of the block: " + t.name; return false; }
        t.nbytes = (size_t)(t.numel() / blck) * bytes;
        t.data = r.take(t.nbytes);
        if (!t.data) { *err = "truncated tensor data: " + t.name; return false; }
        index_[t.name] = tensors_.size();
        tensors_.push_back(t);
    }
    if (!r.ok) { *err = "truncated file"; return false; }
    return true;
}

const GgmlTensor* GgmlFile::find(const std::string& name) const {
    auto it = index_.find(name);
    return it == index_.end() ? nullptr : &tensors_[it->second];
}

// ggml-quants.c dequantize_row_* (block formats of ggml: d / m f16 scale and offset, 4-bit
// nibbles lo = elements 0..15, hi = 16..31 of a block; q5 adds the fifth bit from qh)
bool ggml_dequant_host(int type, const uint8_t* src, int64_t n, float* dst) {
    auto f16 = [](const uint8_t* p) { uint16_t h; memcpy(&h, p, 2); return h2f(h); };
    switch (type) {
        case GG_F32: memcpy(dst, src, n * 4); return true;
        case GG_F16:
            for (int64_t i = 0; i < n; ++i) dst[i] = f16(src + 2 * i);
            return true;
        case GG_Q8_0:
            for (int64_t b = 0; b < n / 32; ++b) {
                const uint8_t* p = src + b * 34;
                const float d = f16(p);
                for (int j = 0; j < 32; ++j) dst[b * 32 + j] = d * (float)(int8_t)p[2 + j];
            }
            return true;
        case GG_Q4_0:
        case GG_Q4_1:
            for (int64_t b = 0; b < n / 32; ++b) {
                const uint8_t* p = src + b * (type == GG_Q4_0 ? 18 : 20);
                const float d = f16(p), m = type == GG_Q4_1 ? f16(p + 2) : 0.0f;
                const uint8_t* qs = p + (type == GG_Q4_0 ? 2 : 4);
                for (int j = 0; j < 16; ++j) {
                    const int lo = qs[j] & 0xf, hi = qs[j] >> 4;
                    if (type == GG_Q4_0) {
                        dst[b * 32 + j] = (float)(lo - 8) * d;
                        dst[b * 32 + j + 16] = (float)(hi - 8) * d;
                    } else {
                        dst[b * 32 + j] = (float)lo * d + m;
                        dst[b * 32 + j + 16] = (float)hi * d + m;
                    }
                }
            }
            return true;
        case GG_Q5_0:
        case GG_Q5_1:
            for (int64_t b = 0; b < n / 32; ++b) {
                const uint8_t* p = src + b * (type == GG_Q5_0 ? 22 : 24);
                const float d = f16(p), m = type == GG_Q5_1 ? f16(p + 2) : 0.0f;
                const uint8_t* q = p + (type == GG_Q5_0 ? 2 : 4);
                uint32_t qh;
                memcpy(&qh, q, 4);
                const uint8_t* qs = q + 4;
                for (int j = 0; j < 16; ++j) {
                    const int x0 = (qs[j] & 0xf) | (((qh >> j) << 4) & 0x10);
                    const int x1 = (qs[j] >> 4) | ((qh >> (j + 12)) & 0x10);
                    if (type == GG_Q5_0) {
                        dst[b * 32 + j] = (float)(x0 - 16) * d;
                        dst[b * 32 + j + 16] = (float)(x1 - 16) * d;
                    } else {
                        dst[b * 32 + j] = (float)x0 * d + m;
                        dst[b * 32 + j + 16] = (float)x1 * d + m;
                    }
                }
            }
            return true;
        default:
            return false;
    }
}

}  // namespace spt
