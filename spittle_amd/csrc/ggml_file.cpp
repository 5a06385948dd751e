// ggml_file.cpp -- see ggml_file.h.  Host side of model loading only: the bulk
// dequantisation of the weight matrices runs on the device (k_init.hip ggml_dequant).
#include "ggml_file.h"
#include "ggml_quant.h"

#include <fcntl.h>
#include <math.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace spt {

namespace {

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

void GgmlFile::type_block(int type, int* blck, int* bytes) { ggml_block_geom(type, blck, bytes); }

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
        // size from an untrusted header: bound the element count by the bytes left in the file
        // before any product can overflow (4 dims of up to 2^31 each)
        const uint64_t max_elems = (uint64_t)(r.end - r.p) / (uint64_t)bytes * (uint64_t)blck;
        uint64_t n_el = 1;
        for (int i = 0; i < t.n_dims; ++i) {
            if ((uint64_t)t.ne[i] > max_elems / n_el) { *err = "truncated tensor data (the header claims more than the file holds): " + t.name; return false; }
            n_el *= (uint64_t)t.ne[i];
        }
        t.nbytes = (size_t)(n_el / blck) * bytes;
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

bool ggml_dequant_host(int type, const uint8_t* src, int64_t n, float* dst) {
    if (type == GQ_F32) {
        memcpy(dst, src, n * 4);
        return true;
    }
    if (type == GQ_F16) {
        for (int64_t i = 0; i < n; ++i) dst[i] = gq_half(src + 2 * i);
        return true;
    }
    int blck, bytes;
    ggml_block_geom(type, &blck, &bytes);
    if (!blck || n % blck) return false;
    for (int64_t b = 0; b < n / blck; ++b) {
        float* o = dst + b * blck;
        ggml_dequant_block(type, src + b * bytes, [o](int i, float v) { o[i] = v; });
    }
    return true;
}

}  // namespace spt
