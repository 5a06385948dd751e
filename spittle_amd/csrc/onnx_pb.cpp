// onnx_pb.cpp -- see onnx_pb.h.  Field numbers follow onnx/onnx.proto (ModelProto.graph = 7;
// GraphProto.node = 1, initializer = 5; NodeProto.input = 1, output = 2, name = 3, op_type = 4,
// attribute = 5, domain = 7; TensorProto.dims = 1, data_type = 2, float_data = 4, int32_data = 5,
// int64_data = 7, name = 8, raw_data = 9, double_data = 10, external_data = 13, data_location = 14;
// AttributeProto.name = 1, f = 2, i = 3, s = 4, ints = 8).
#include "onnx_pb.h"

#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>

namespace spt {
namespace onnx {

namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;

    bool done() const { return !ok || p >= end; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int s = 0; s < 64; s += 7) {
            if (p >= end) { ok = false; return 0; }
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    // one field: tag, and for length-delimited fields the payload's bounds
    bool field(uint32_t* num, int* wt, Reader* sub) {
        const uint64_t tag = varint();
        if (!ok) return false;
        *num = (uint32_t)(tag >> 3);
        *wt = (int)(tag & 7);
        switch (*wt) {
            case 0: sub->p = p; varint(); sub->end = p; return ok;
            case 1: if (end - p < 8) return ok = false; sub->p = p; p += 8; sub->end = p; return true;
            case 5: if (end - p < 4) return ok = false; sub->p = p; p += 4; sub->end = p; return true;
            case 2: {
                const uint64_t n = varint();
                if (!ok || n > (uint64_t)(end - p)) return ok = false;
                sub->p = p; p += n; sub->end = p;
                return true;
            }
            default: return ok = false;  // groups (3, 4) are not used by ONNX
        }
    }
};

uint64_t as_varint(const Reader& r) {
    Reader t = r;
    return t.varint();
}
std::string as_string(const Reader& r) { return std::string((const char*)r.p, (size_t)(r.end - r.p)); }
// a fixed32 float: only from a wire-type-5 field (exactly 4 payload bytes); anything else is a
// malformed file, not 4 bytes read past a shorter field
bool as_f32(int wt, const Reader& r, float* f) {
    if (wt != 5 || r.end - r.p != 4) return false;
    memcpy(f, r.p, 4);
    return true;
}

// repeated scalar fields, packed (wire type 2) or not; a wrong wire type fails the parse
bool rep_varint(int wt, const Reader& r, std::vector<int64_t>* out) {
    if (wt == 0) { out->push_back((int64_t)as_varint(r)); return true; }
    if (wt != 2) return false;
    Reader t = r;
    while (!t.done()) out->push_back((int64_t)t.varint());
    return t.ok;
}
bool rep_f32(int wt, const Reader& r, std::vector<float>* out) {
    if (wt == 5) {
        float f;
        if (!as_f32(wt, r, &f)) return false;
        out->push_back(f);
        return true;
    }
    if (wt != 2 || (r.end - r.p) % 4) return false;
    for (const uint8_t* q = r.p; q + 4 <= r.end; q += 4) {
        float f;
        memcpy(&f, q, 4);
        out->push_back(f);
    }
    return true;
}

bool parse_tensor(Reader r, Tensor* t) {
    uint32_t num; int wt; Reader s{};
    bool external = false;
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) return false;
        switch (num) {
            case 1: if (!rep_varint(wt, s, &t->dims)) return false; break;
            case 2: if (wt != 0) return false; t->data_type = (int)as_varint(s); break;
            case 4: if (!rep_f32(wt, s, &t->f32)) return false; break;
            case 5: case 7: if (!rep_varint(wt, s, &t->i64)) return false; break;
            case 8: t->name = as_string(s); break;
            case 9: t->raw = s.p; t->raw_len = (size_t)(s.end - s.p); break;
            case 10: {  // double_data: fixed64, packed or not
                if (wt == 1) { double d; memcpy(&d, s.p, 8); t->f32.push_back((float)d); }  // field() gave 8 bytes
                else if (wt != 2 || (s.end - s.p) % 8) return false;
                else for (const uint8_t* q = s.p; q + 8 <= s.end; q += 8) { double d; memcpy(&d, q, 8); t->f32.push_back((float)d); }
                break;
            }
            case 13: {  // StringStringEntryProto {key = 1, value = 2}
                Reader e = s; std::string k, v; uint32_t n2; int w2; Reader s2{};
                while (!e.done()) {
                    if (!e.field(&n2, &w2, &s2)) return false;
                    if (n2 == 1) k = as_string(s2);
                    else if (n2 == 2) v = as_string(s2);
                }
                if (k == "location") t->ext_location = v;
                else if (k == "offset") t->ext_offset = strtoll(v.c_str(), nullptr, 10);
                else if (k == "length") t->ext_length = strtoll(v.c_str(), nullptr, 10);
                break;
            }
            case 14: if (wt != 0) return false; external = as_varint(s) == 1; break;
            default: break;
        }
    }
    if (external && t->ext_location.empty()) return false;
    if (!external) t->ext_location.clear();
    // each extent and their product bounded (2^34 elements = 64 GiB of f32): no wrapped int64
    // reaches Tensor::numel / to_f32's resize
    int64_t n = 1;
    for (int64_t d : t->dims) {
        if (d < 0 || d > (int64_t)1 << 34) return false;
        if (d > 0 && n > (((int64_t)1 << 34) / d)) return false;
        n *= d;
    }
    return true;
}

bool parse_graph(Reader r, Graph* g, int depth);

bool parse_attr(Reader r, Attribute* a, int depth) {
    uint32_t num; int wt; Reader s{};
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) return false;
        switch (num) {
            case 1: a->name = as_string(s); break;
            case 2: if (!as_f32(wt, s, &a->f)) return false; break;
            case 3: if (wt != 0) return false; a->i = (int64_t)as_varint(s); break;
            case 4: a->s = as_string(s); break;
            case 6:
                if (depth > 8) return false;  // nested subgraphs: bounded
                a->g = std::make_shared<Graph>();
                if (!parse_graph(s, a->g.get(), depth + 1)) return false;
                break;
            case 8: if (!rep_varint(wt, s, &a->ints)) return false; break;
            default: break;
        }
    }
    return true;
}

bool parse_node(Reader r, Node* n, int depth) {
    uint32_t num; int wt; Reader s{};
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) return false;
        switch (num) {
            case 1: n->inputs.push_back(as_string(s)); break;
            case 2: n->outputs.push_back(as_string(s)); break;
            case 3: n->name = as_string(s); break;
            case 4: n->op_type = as_string(s); break;
            case 5: { Attribute a; if (!parse_attr(s, &a, depth)) return false; n->attrs.push_back(a); break; }
            case 7: n->domain = as_string(s); break;
            default: break;
        }
    }
    return true;
}

// ValueInfoProto {name = 1}
std::string value_info_name(Reader r) {
    uint32_t num; int wt; Reader s{};
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) break;
        if (num == 1) return as_string(s);
    }
    return std::string();
}

bool parse_graph(Reader r, Graph* g, int depth) {
    uint32_t num; int wt; Reader s{};
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) return false;
        if (num == 1 && wt == 2) {
            Node n;
            if (!parse_node(s, &n, depth)) return false;
            g->nodes.push_back(std::move(n));
        } else if (num == 5 && wt == 2) {
            Tensor t;
            if (!parse_tensor(s, &t)) return false;
            g->initializers.push_back(std::move(t));
        } else if (num == 12 && wt == 2) {
            g->outputs.push_back(value_info_name(s));
        }
    }
    return r.ok;
}

float half_to_f32(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1F, m = h & 0x3FF;
    uint32_t u;
    if (e == 0) {
        if (m == 0) u = s;
        else {  // subnormal
            float f = std::ldexp((float)m, -24);
            return s ? -f : f;
        }
    } else if (e == 31) {
        u = s | 0x7F800000u | (m << 13);
    } else {
        u = s | ((e + 112) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

bool map_file(const std::string& path, const uint8_t** p, size_t* len, std::string* err) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) { *err = "cannot open " + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) { ::close(fd); *err = "cannot stat " + path; return false; }
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) { *err = "cannot map " + path; return false; }
    *p = (const uint8_t*)m;
    *len = (size_t)st.st_size;
    return true;
}

}  // namespace

int64_t Tensor::numel() const {
    int64_t n = 1;
    for (int64_t d : dims) n *= d;
    return n;
}

bool Tensor::to_f32(std::vector<float>* out, std::string* err) const {
    const int64_t n = numel();
    out->resize((size_t)n);
    auto need = [&](size_t esz) {
        if (raw && raw_len != (size_t)n * esz) {
            *err = "tensor '" + name + "': raw_data size does not match its dims";
            return false;
        }
        if (!raw && ((esz == 4 && data_type == T_FLOAT) ? f32.size() : i64.size()) != (size_t)n &&
            !(data_type == T_DOUBLE && f32.size() == (size_t)n)) {
            *err = "tensor '" + name + "': element count does not match its dims";
            return false;
        }
        return true;
    };
    switch (data_type) {
        case T_FLOAT:
            if (!need(4)) return false;
            if (raw) memcpy(out->data(), raw, (size_t)n * 4);
            else *out = f32;
            return true;
        case T_DOUBLE:
            if (raw) {
                if (raw_len != (size_t)n * 8) { *err = "tensor '" + name + "': raw_data size does not match its dims"; return false; }
                for (int64_t i = 0; i < n; ++i) { double d; memcpy(&d, raw + 8 * i, 8); (*out)[i] = (float)d; }
            } else {
                if (f32.size() != (size_t)n) { *err = "tensor '" + name + "': element count does not match its dims"; return false; }
                *out = f32;
            }
            return true;
        case T_FLOAT16: case T_BFLOAT16:
            if (!need(2)) return false;
            for (int64_t i = 0; i < n; ++i) {
                uint16_t h;
                if (raw) memcpy(&h, raw + 2 * i, 2);
                else h = (uint16_t)i64[i];
                if (data_type == T_FLOAT16) (*out)[i] = half_to_f32(h);
                else { const uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); (*out)[i] = f; }
            }
            return true;
        case T_INT8: case T_UINT8:
            if (!need(1)) return false;
            for (int64_t i = 0; i < n; ++i)
                (*out)[i] = raw ? (data_type == T_INT8 ? (float)(int8_t)raw[i] : (float)raw[i])
                                : (float)(data_type == T_INT8 ? (int64_t)(int8_t)i64[i] : (int64_t)(uint8_t)i64[i]);
            return true;
        case T_INT32: case T_INT64: {
            const size_t esz = data_type == T_INT32 ? 4 : 8;
            if (!need(esz)) return false;
            for (int64_t i = 0; i < n; ++i) {
                int64_t v;
                if (raw) {
                    if (esz == 4) { int32_t w; memcpy(&w, raw + 4 * i, 4); v = w; }
                    else memcpy(&v, raw + 8 * i, 8);
                } else v = i64[i];
                (*out)[i] = (float)v;
            }
            return true;
        }
        default:
            *err = "tensor '" + name + "': unsupported data type " + std::to_string(data_type);
            return false;
    }
}

const Attribute* Node::attr(const std::string& n) const {
    for (const Attribute& a : attrs)
        if (a.name == n) return &a;
    return nullptr;
}

bool Model::open(const std::string& path, std::string* err) {
    path_ = path;
    if (!map_file(path, &map_, &len_, err)) return false;
    Reader r{map_, map_ + len_};
    uint32_t num; int wt; Reader s{};
    bool have_graph = false;
    while (!r.done()) {
        if (!r.field(&num, &wt, &s)) break;
        if (num == 7 && wt == 2) {
            if (!parse_graph(s, &graph_, 0)) { *err = path + ": malformed GraphProto"; return false; }
            have_graph = true;
        }
    }
    if (!r.ok) { *err = path + ": malformed protobuf (not an ONNX model?)"; return false; }
    if (!have_graph) { *err = path + ": no graph in the model"; return false; }
    return resolve_external(err);
}

bool Model::resolve_external(std::string* err) {
    const size_t slash = path_.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "." : path_.substr(0, slash);
    std::map<std::string, size_t> opened;
    for (Tensor& t : graph_.initializers) {
        if (t.ext_location.empty()) continue;
        if (t.ext_location.find("..") != std::string::npos || t.ext_location[0] == '/') {
            *err = "tensor '" + t.name + "': external data outside the model directory";
            return false;
        }
        auto it = opened.find(t.ext_location);
        if (it == opened.end()) {
            const uint8_t* p; size_t len;
            if (!map_file(dir + "/" + t.ext_location, &p, &len, err)) return false;
            ext_maps_.push_back({p, len});
            it = opened.emplace(t.ext_location, ext_maps_.size() - 1).first;
        }
        const auto& m = ext_maps_[it->second];
        const int64_t len = t.ext_length >= 0 ? t.ext_length : (int64_t)m.second - t.ext_offset;
        if (t.ext_offset < 0 || len < 0 || (uint64_t)t.ext_offset + (uint64_t)len > m.second) {
            *err = "tensor '" + t.name + "': external data range outside its file";
            return false;
        }
        t.raw = m.first + t.ext_offset;
        t.raw_len = (size_t)len;
    }
    return true;
}

Model::~Model() {
    if (map_) munmap((void*)map_, len_);
    for (auto& m : ext_maps_) munmap((void*)m.first, m.second);
}

}  // namespace onnx
}  // namespace spt
