// pk_onnx.cpp -- the Parakeet-V3 ONNX model directory -> the engine's tensor table (see pk_onnx.h).
//
// The export is torch.onnx's of NeMo's FastConformer-TDT modules, dynamically quantised to int8 by
// ONNX Runtime [upstream, recalled; no export exists offline, so this is unpinned against the real
// file].  What the loader relies on, each the documented behaviour of those tools:
//   * node names carry the module path ("/layers.0/feed_forward1/linear1/MatMul"), so a weight's
//     role follows from the node that consumes it, whatever the initializer is called (torch names
//     transposed Linear weights "onnx::MatMul_<n>");
//   * a quantised weight W is the initializer triple W_quantized / W_scale / W_zero_point
//     (quantize_dynamic; per tensor or per output channel) or a DequantizeLinear node (QDQ form):
//     value = (q - zero_point) * scale;
//   * MatMul weights are [K][N] (x . W), Gemm weights follow transB, Conv weights are
//     [out][in / group][k...] as in torch, LSTM weights are ONNX [1][4H][in] with gates (i, o, f, c)
//     (DynamicQuantizeLSTM: [1][in][4H]) -- torch's nn.LSTM is (i, f, g, o);
//   * parameters used as they are (biases, LayerNorm scale / shift, pos_bias_u / v, BatchNorm
//     statistics) keep their state-dict names, which are used when they match the NeMo key table
//     (spittle_amd/parakeet.py nemo_key_map); BatchNorm folded into the depthwise convolution is
//     accepted (the engine's BatchNorm is then the identity).
#include "pk_onnx.h"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <fstream>
#include <set>
#include <sstream>

#include "onnx_pb.h"

namespace spt {

namespace {

struct Val {
    std::vector<int64_t> dims;
    std::vector<float> v;
};

std::vector<std::string> tokens(const std::string& s) {
    std::vector<std::string> t;
    std::string cur;
    for (char c : s) {
        if (c == '.' || c == '/' || c == ':') {
            if (!cur.empty()) t.push_back(cur);
            cur.clear();
        } else cur += c;
    }
    if (!cur.empty()) t.push_back(cur);
    return t;
}

// canonical module path: separators unified, consecutive duplicate components dropped
// ("joint/joint_net/joint_net.2" -> joint.joint_net.2), a leading "encoder" / "model" dropped
std::string canon(const std::string& s) {
    std::vector<std::string> t = tokens(s), o;
    for (const std::string& x : t)
        if (o.empty() || o.back() != x) o.push_back(x);
    while (!o.empty() && (o[0] == "encoder" || o[0] == "model" || o[0] == "onnx")) o.erase(o.begin());
    std::string r;
    for (const std::string& x : o) r += (r.empty() ? "" : ".") + x;
    return r;
}

// the module path of a node: its name without the last component (the op)
std::string node_path(const onnx::Node& n) {
    const size_t k = n.name.find_last_of('/');
    return k == std::string::npos ? std::string() : canon(n.name.substr(0, k));
}

// NeMo state-dict key (canonical, "encoder." dropped) -> engine tensor id (oracle/po_model.c table)
std::map<std::string, int> key_table(int max_layers) {
    std::map<std::string, int> m;
    const std::pair<int, const char*> pre[] = {{1, "conv.0"}, {3, "conv.2"}, {5, "conv.3"}, {7, "conv.5"},
                                               {9, "conv.6"}, {11, "out"}};
    for (auto& p : pre) {
        m[canon(std::string("pre_encode.") + p.second + ".weight")] = p.first;
        m[canon(std::string("pre_encode.") + p.second + ".bias")] = p.first + 1;
    }
    const std::pair<const char*, int> names[] = {
        {"norm_feed_forward1", 0}, {"feed_forward1.linear1", 2}, {"feed_forward1.linear2", 4}, {"norm_self_att", 6},
        {"self_attn.linear_q", 8}, {"self_attn.linear_k", 10}, {"self_attn.linear_v", 12}, {"self_attn.linear_out", 14},
        {"norm_conv", 19}, {"conv.pointwise_conv1", 21}, {"conv.depthwise_conv", 23}, {"conv.pointwise_conv2", 29},
        {"norm_feed_forward2", 31}, {"feed_forward2.linear1", 33}, {"feed_forward2.linear2", 35}, {"norm_out", 37}};
    for (int l = 0; l < max_layers; ++l) {
        const int b = 1000 + 64 * l;
        const std::string p = "layers." + std::to_string(l) + ".";
        for (auto& n : names) {
            m[canon(p + n.first + ".weight")] = b + n.second;
            m[canon(p + n.first + ".bias")] = b + n.second + 1;
        }
        m[canon(p + "self_attn.linear_pos.weight")] = b + 16;
        m[canon(p + "self_attn.pos_bias_u")] = b + 17;
        m[canon(p + "self_attn.pos_bias_v")] = b + 18;
        const std::pair<const char*, int> bn[] = {{"weight", 25}, {"bias", 26}, {"running_mean", 27}, {"running_var", 28}};
        for (auto& x : bn) m[canon(p + "conv.batch_norm." + x.first)] = b + x.second;
    }
    m[canon("decoder.prediction.embed.weight")] = 90000;
    const std::pair<const char*, int> jn[] = {{"joint.enc", 90009}, {"joint.pred", 90011}, {"joint.joint_net.2", 90013}};
    for (auto& x : jn) {
        m[canon(std::string(x.first) + ".weight")] = x.second;
        m[canon(std::string(x.first) + ".bias")] = x.second + 1;
    }
    return m;
}

struct Mapper {
    std::map<std::string, int> keys = key_table(64);
    std::map<int, Val>* out;
    std::set<int> assigned;
    std::string graph_name;

    // exact canonical match, else the unique known key the candidate is a token-suffix of
    int lookup(const std::string& cand_raw) const {
        const std::string c = canon(cand_raw);
        if (c.empty()) return -1;
        auto it = keys.find(c);
        if (it != keys.end()) return it->second;
        int hit = -1;
        for (auto& kv : keys) {
            const std::string& k = kv.first;
            if (k.size() > c.size() && k.compare(k.size() - c.size(), c.size(), c) == 0 && k[k.size() - c.size() - 1] == '.') {
                if (hit >= 0 && hit != kv.second) return -2;  // ambiguous
                hit = kv.second;
            }
        }
        return hit;
    }
    // a tensor id takes one value: the same value again (a weight consumed by two nodes) is
    // accepted, a different one means the graph maps two tensors onto one role -- an error, not a
    // silent first-wins choice
    bool put(int tid, Val v, std::string* err, const std::string& what) {
        if (tid == -2) { *err = "node '" + what + "': its parameter matches several tensors"; return false; }
        if (tid < 0) return true;
        if (assigned.count(tid)) {
            const Val& o = (*out)[tid];
            if (o.dims == v.dims && o.v == v.v) return true;
            *err = "node '" + what + "': a second, different value for " + pk_tensor_name(tid);
            return false;
        }
        assigned.insert(tid);
        (*out)[tid] = std::move(v);
        return true;
    }
};

Val transpose2(const Val& a) {
    Val t;
    const int64_t R = a.dims[0], C = a.dims[1];
    t.dims = {C, R};
    t.v.resize(a.v.size());
    for (int64_t r = 0; r < R; ++r)
        for (int64_t c = 0; c < C; ++c) t.v[(size_t)c * R + r] = a.v[(size_t)r * C + c];
    return t;
}

// (q - zp) * scale, per tensor or per channel along the axis whose length matches the scale's
bool dequant(const onnx::Tensor& q, const onnx::Tensor& sc, const onnx::Tensor* zp, Val* out, std::string* err) {
    std::vector<float> qv, s, z;
    if (!q.to_f32(&qv, err) || !sc.to_f32(&s, err)) return false;
    if (zp && !zp->to_f32(&z, err)) return false;
    if (z.empty()) z.assign(s.size(), 0.f);
    if (z.size() != s.size() || s.empty()) { *err = "quantised tensor '" + q.name + "': scale / zero point sizes differ"; return false; }
    out->dims = q.dims;
    out->v.resize(qv.size());
    if (s.size() == 1) {
        for (size_t i = 0; i < qv.size(); ++i) out->v[i] = (qv[i] - z[0]) * s[0];
        return true;
    }
    // per channel: the output-channel axis -- the last of a MatMul weight [K][N], the first of a
    // convolution weight [out][in / group][k...] -- or else the axis whose extent matches
    int axis = -1;
    const int rank = (int)q.dims.size();
    if (rank == 2 && q.dims[1] == (int64_t)s.size()) axis = 1;
    else if (rank >= 3 && q.dims[0] == (int64_t)s.size()) axis = 0;
    for (int a = rank - 1; axis < 0 && a >= 0; --a)
        if (q.dims[a] == (int64_t)s.size()) axis = a;
    if (axis < 0) { *err = "quantised tensor '" + q.name + "': no axis matches its " + std::to_string(s.size()) + " scales"; return false; }
    int64_t inner = 1;
    for (size_t a = axis + 1; a < q.dims.size(); ++a) inner *= q.dims[a];
    for (size_t i = 0; i < qv.size(); ++i) {
        const size_t c = (size_t)((int64_t)i / inner % (int64_t)s.size());
        out->v[i] = (qv[i] - z[c]) * s[c];
    }
    return true;
}

bool file_exists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

std::string pick(const std::string& dir, const char* stem) {
    for (const char* suf : {".int8.onnx", ".onnx"}) {  // ParakeetModelParams::int8(): the quantised export first
        const std::string p = dir + "/" + stem + suf;
        if (file_exists(p)) return p;
    }
    return std::string();
}

// every initializer as f32, quantised triples and DequantizeLinear outputs dequantised
bool values(const onnx::Model& m, std::map<std::string, Val>* vals, int* n_q, std::string* err) {
    std::map<std::string, const onnx::Tensor*> init;
    for (const onnx::Tensor& t : m.graph().initializers) init[t.name] = &t;
    for (const onnx::Tensor& t : m.graph().initializers) {
        const std::string suf = "_quantized";
        if (t.name.size() > suf.size() && t.name.compare(t.name.size() - suf.size(), suf.size(), suf) == 0) {
            const std::string base = t.name.substr(0, t.name.size() - suf.size());
            auto s = init.find(base + "_scale");
            if (s != init.end()) {
                auto z = init.find(base + "_zero_point");
                Val v;
                if (!dequant(t, *s->second, z == init.end() ? nullptr : z->second, &v, err)) return false;
                (*vals)[base] = v;
                (*vals)[t.name] = std::move(v);
                ++*n_q;
                continue;
            }
        }
        if (t.data_type == onnx::T_FLOAT || t.data_type == onnx::T_FLOAT16 || t.data_type == onnx::T_BFLOAT16 ||
            t.data_type == onnx::T_DOUBLE || t.data_type == onnx::T_INT8 || t.data_type == onnx::T_UINT8) {
            Val v;
            v.dims = t.dims;
            if (!t.to_f32(&v.v, err)) return false;
            (*vals)[t.name] = std::move(v);
        }
    }
    for (const onnx::Node& n : m.graph().nodes) {  // QDQ form
        if (n.op_type != "DequantizeLinear" || n.inputs.size() < 2 || n.outputs.empty()) continue;
        auto q = init.find(n.inputs[0]);
        auto s = init.find(n.inputs[1]);
        if (q == init.end() || s == init.end()) continue;
        const onnx::Tensor* z = n.inputs.size() > 2 ? (init.count(n.inputs[2]) ? init[n.inputs[2]] : nullptr) : nullptr;
        Val v;
        if (!dequant(*q->second, *s->second, z, &v, err)) return false;
        (*vals)[n.outputs[0]] = std::move(v);
        ++*n_q;
    }
    return true;
}

const Val* find_val(const std::map<std::string, Val>& vals, const std::string& name) {
    auto it = vals.find(name);
    return it == vals.end() ? nullptr : &it->second;
}

// ONNX LSTM gate blocks (i, o, f, c) -> torch (i, f, g, o)
Val lstm_gates(const float* src, int64_t H, int64_t cols) {
    static const int perm[4] = {0, 2, 3, 1};
    Val v;
    v.dims = {4 * H, cols};
    v.v.resize((size_t)(4 * H * cols));
    for (int q = 0; q < 4; ++q)
        std::copy(src + (size_t)perm[q] * H * cols, src + (size_t)(perm[q] + 1) * H * cols, v.v.begin() + (size_t)q * H * cols);
    return v;
}

bool map_graph(const onnx::Model& m, Mapper* mp, int* n_q, std::string* err) {
#define PUT(...) do { if (!mp->put(__VA_ARGS__)) return false; } while (0)
    std::map<std::string, Val> vals;
    if (!values(m, &vals, n_q, err)) return false;
    std::map<std::string, int> bias_uv;  // per self_attn path: pos_bias Adds seen (u, then v)
    int lstm_layer = 0;
    for (const onnx::Node& n : m.graph().nodes) {
        const std::string path = node_path(n);
        const std::string& op = n.op_type;
        auto in = [&](size_t i) -> const Val* { return i < n.inputs.size() ? find_val(vals, n.inputs[i]) : nullptr; };
        if (op == "MatMul" || op == "MatMulInteger" || op == "MatMulIntegerToFloat") {
            const Val* w = in(1);
            if (w && w->dims.size() == 2) PUT(mp->lookup(path + ".weight"), transpose2(*w), err, n.name);
        } else if (op == "Gemm") {
            const onnx::Attribute* tb = n.attr("transB");
            if (const Val* w = in(1); w && w->dims.size() == 2)
                PUT(mp->lookup(path + ".weight"), tb && tb->i ? *w : transpose2(*w), err, n.name);
            if (const Val* b = in(2)) PUT(mp->lookup(path + ".bias"), *b, err, n.name);
        } else if (op == "Conv" || op == "ConvInteger") {
            if (const Val* w = in(1)) PUT(mp->lookup(path + ".weight"), *w, err, n.name);
            if (op == "Conv")
                if (const Val* b = in(2)) PUT(mp->lookup(path + ".bias"), *b, err, n.name);
        } else if (op == "LayerNormalization") {
            if (const Val* w = in(1)) PUT(mp->lookup(path + ".weight"), *w, err, n.name);
            if (const Val* b = in(2)) PUT(mp->lookup(path + ".bias"), *b, err, n.name);
        } else if (op == "BatchNormalization") {
            const char* f[4] = {".weight", ".bias", ".running_mean", ".running_var"};
            for (int i = 0; i < 4; ++i)
                if (const Val* v = in(1 + i)) PUT(mp->lookup(path + f[i]), *v, err, n.name);
        } else if (op == "Gather") {
            const Val* w = in(0);
            if (w && w->dims.size() == 2) PUT(mp->lookup(path + ".weight"), *w, err, n.name);
        } else if (op == "Add" || op == "Sub") {
            for (size_t i = 0; i < n.inputs.size(); ++i) {
                const Val* v = in(i);
                if (!v) continue;
                int tid = mp->lookup(n.inputs[i]);  // a parameter used as it is keeps its name
                if (tid == -2) tid = -1;            // a generic initializer name is no role
                if (tid < 0 && v->dims.size() == 2 && path.size() >= 9 && path.compare(path.size() - 9, 9, "self_attn") == 0) {
                    // unnamed [H][dk] operands of the relative attention: pos_bias_u, then pos_bias_v
                    const int k = bias_uv[path]++;
                    if (k >= 2) {
                        *err = "node '" + n.name + "': a third unnamed [H][dk] Add operand in " + path +
                               " (only pos_bias_u then pos_bias_v are expected)";
                        return false;
                    }
                    tid = mp->lookup(path + (k == 0 ? ".pos_bias_u" : ".pos_bias_v"));
                }
                if (tid < 0 && v->dims.size() == 1) tid = mp->lookup(path + ".bias");
                PUT(tid, *v, err, n.name);
            }
        } else if (op == "LSTM" || op == "DynamicQuantizeLSTM") {
            const Val* W = in(1);
            const Val* R = in(2);
            const Val* B = in(3);
            if (!W || !R || W->dims.size() != 3 || R->dims.size() != 3) {
                *err = "LSTM node '" + n.name + "': weights are not initializers";
                return false;
            }
            Val w = *W, r = *R;
            if (op == "DynamicQuantizeLSTM") {  // [1][in][4H] -> [1][4H][in]
                Val w2{{w.dims[1], w.dims[2]}, w.v}, r2{{r.dims[1], r.dims[2]}, r.v};
                w2 = transpose2(w2); r2 = transpose2(r2);
                w = Val{{1, w2.dims[0], w2.dims[1]}, w2.v};
                r = Val{{1, r2.dims[0], r2.dims[1]}, r2.v};
            }
            const int64_t H4 = w.dims[1], H = H4 / 4, IN = w.dims[2];
            if (H4 % 4 || r.dims[1] != H4 || r.dims[2] != H) { *err = "LSTM node '" + n.name + "': bad weight shapes"; return false; }
            const int base = 90001 + 4 * lstm_layer;
            PUT(base + 0, lstm_gates(w.v.data(), H, IN), err, n.name);
            PUT(base + 1, lstm_gates(r.v.data(), H, H), err, n.name);
            Val bi, bh;
            if (B && (int64_t)B->v.size() == 8 * H) {
                bi = lstm_gates(B->v.data(), H, 1);
                bh = lstm_gates(B->v.data() + 4 * H, H, 1);
            } else {
                bi.v.assign((size_t)(4 * H), 0.f);
                bh.v.assign((size_t)(4 * H), 0.f);
            }
            bi.dims = {4 * H}; bh.dims = {4 * H};
            PUT(base + 2, bi, err, n.name);
            PUT(base + 3, bh, err, n.name);
            ++lstm_layer;
        }
    }
    // parameters consumed by ops the node pass does not know keep their state-dict names
    for (auto& kv : vals) {
        const int tid = mp->lookup(kv.first);
        if (tid >= 0 && !mp->assigned.count(tid)) PUT(tid, kv.second, err, kv.first);
    }
    return true;
}

bool read_vocab(const std::string& path, int n_vocab, std::vector<std::string>* pieces, std::string* err) {
    std::ifstream f(path);
    if (!f) { *err = "cannot read " + path; return false; }
    pieces->assign((size_t)n_vocab, std::string());
    std::vector<bool> seen((size_t)n_vocab, false);
    std::string line;
    int n_set = 0;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const size_t sp = line.find_last_of(' ');
        if (sp == std::string::npos) continue;
        char* end = nullptr;
        const long id = strtol(line.c_str() + sp + 1, &end, 10);
        if (!end || *end) continue;
        if (id < 0 || id > n_vocab) { *err = path + ": token id " + std::to_string(id) + " out of range"; return false; }
        if (id == n_vocab) continue;  // the blank (<blk>)
        if (!seen[id]) ++n_set;
        seen[id] = true;
        (*pieces)[id] = line.substr(0, sp);
    }
    if (n_set != n_vocab) {
        *err = path + ": " + std::to_string(n_set) + " of " + std::to_string(n_vocab) + " token ids present";
        return false;
    }
    return true;
}

}  // namespace

std::string pk_tensor_name(int tid) {
    if (tid >= 90001 && tid <= 90008) {
        static const char* nm[4] = {"weight_ih", "weight_hh", "bias_ih", "bias_hh"};
        return "decoder.prediction.dec_rnn.lstm." + std::string(nm[(tid - 90001) % 4]) + "_l" + std::to_string((tid - 90001) / 4);
    }
    for (auto& kv : key_table(64))
        if (kv.second == tid) return (tid < 90000 ? "encoder." : "") + kv.first;
    return "tensor " + std::to_string(tid);
}

bool is_parakeet_onnx_dir(const std::string& path) {
    struct stat st;
    if (stat(path.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return false;
    return !pick(path, "encoder-model").empty();
}

bool load_parakeet_onnx(const std::string& dir, PkOnnxModel* out, std::string* err) {
    out->encoder_file = pick(dir, "encoder-model");
    out->decoder_file = pick(dir, "decoder_joint-model");
    if (out->encoder_file.empty() || out->decoder_file.empty()) {
        *err = dir + ": expected encoder-model[.int8].onnx and decoder_joint-model[.int8].onnx (the onnx-asr export)";
        return false;
    }
    std::map<int, Val> t;
    Mapper mp;
    mp.out = &t;
    {
        onnx::Model enc;
        if (!enc.open(out->encoder_file, err) || !map_graph(enc, &mp, &out->n_quantized, err)) return false;
    }
    {
        onnx::Model dec;
        if (!dec.open(out->decoder_file, err) || !map_graph(dec, &mp, &out->n_quantized, err)) return false;
    }
    // dimensions from the tensors themselves
    auto need = [&](int tid, size_t rank, const char* what) -> const Val* {
        auto it = t.find(tid);
        if (it == t.end()) { *err = std::string("model has no ") + what; return nullptr; }
        if (it->second.dims.size() < rank) { *err = std::string(what) + ": unexpected rank"; return nullptr; }
        return &it->second;
    };
    PkDims d;
    d.name = "onnx:" + dir;
    const Val* c0 = need(1, 1, "subsampling conv.0 weight");
    const Val* lin = need(11, 2, "subsampling output linear weight");
    const Val* ff1 = need(1002, 2, "layer-0 feed-forward weight");
    const Val* pbu = need(1017, 2, "layer-0 pos_bias_u");
    const Val* dw = need(1023, 1, "layer-0 depthwise convolution weight");
    const Val* emb = need(90000, 2, "prediction-network embedding");
    const Val* jo = need(90013, 2, "joint output weight");
    if (!c0 || !lin || !ff1 || !pbu || !dw || !emb || !jo) return false;
    d.sub_ch = (int)c0->dims[0];
    d.d = (int)lin->dims[0];
    const int F3 = (int)(lin->dims[1] / d.sub_ch);
    d.n_mels = F3 * 8;  // three stride-2 halvings of the mel axis (nemo128: 128 -> 16)
    d.ff = (int)ff1->dims[0];
    d.n_heads = (int)pbu->dims[0];
    d.conv_k = (int)dw->dims.back();
    d.pred = (int)emb->dims[1];
    d.n_vocab = (int)emb->dims[0] - 1;
    d.n_dur = (int)jo->dims[0] - d.n_vocab - 1;
    d.n_layers = 0;
    while (t.count(1000 + 64 * d.n_layers + 2)) ++d.n_layers;
    if (d.n_layers < 1 || d.n_dur < 1 || d.n_vocab < 1) { *err = "inconsistent model dimensions"; return false; }
    // BatchNorm folded into the depthwise convolution: the engine's BatchNorm is the identity
    for (int l = 0; l < d.n_layers; ++l) {
        const int b = 1000 + 64 * l;
        if (!t.count(b + 25) && !t.count(b + 26) && !t.count(b + 27) && !t.count(b + 28)) {
            t[b + 25] = Val{{(int64_t)d.d}, std::vector<float>((size_t)d.d, 1.f)};
            t[b + 26] = Val{{(int64_t)d.d}, std::vector<float>((size_t)d.d, 0.f)};
            t[b + 27] = Val{{(int64_t)d.d}, std::vector<float>((size_t)d.d, 0.f)};
            t[b + 28] = Val{{(int64_t)d.d}, std::vector<float>((size_t)d.d, 1.f - 1e-5f)};  // 1 / sqrt(var + eps) = 1
        }
        if (!t.count(b + 24)) t[b + 24] = Val{{(int64_t)d.d}, std::vector<float>((size_t)d.d, 0.f)};  // no conv bias
    }
    // every tensor in its NeMo shape: the leading (output) extent and the product of the rest, so a
    // weight mapped in the wrong orientation fails here rather than loading with the right element
    // count (square d x d projections cannot be told apart by shape)
    {
        const int64_t D = d.d, C = d.sub_ch, FF = d.ff, P = d.pred, F3 = d.n_mels / 8;
        const int64_t NO = d.n_vocab + 1 + d.n_dur, dk = D / std::max(1, d.n_heads);
        std::map<int, std::pair<int64_t, int64_t>> want = {
            {1, {C, 9}}, {2, {C, 1}}, {3, {C, 9}}, {4, {C, 1}}, {5, {C, C}}, {6, {C, 1}}, {7, {C, 9}}, {8, {C, 1}},
            {9, {C, C}}, {10, {C, 1}}, {11, {D, C * F3}}, {12, {D, 1}},
            {90000, {d.n_vocab + 1, P}}, {90009, {P, D}}, {90010, {P, 1}}, {90011, {P, P}}, {90012, {P, 1}},
            {90013, {NO, P}}, {90014, {NO, 1}}};
        for (int j = 0; j < 2; ++j) {
            want[90001 + 4 * j] = {4 * P, P};
            want[90002 + 4 * j] = {4 * P, P};
            want[90003 + 4 * j] = {4 * P, 1};
            want[90004 + 4 * j] = {4 * P, 1};
        }
        for (int l = 0; l < d.n_layers; ++l) {
            const int b = 1000 + 64 * l;
            const std::pair<int, std::pair<int64_t, int64_t>> lw[] = {
                {2, {FF, D}}, {3, {FF, 1}}, {4, {D, FF}}, {8, {D, D}}, {10, {D, D}}, {12, {D, D}}, {14, {D, D}},
                {16, {D, D}}, {17, {d.n_heads, dk}}, {18, {d.n_heads, dk}}, {21, {2 * D, D}}, {22, {2 * D, 1}},
                {23, {D, d.conv_k}}, {29, {D, D}}, {33, {FF, D}}, {34, {FF, 1}}, {35, {D, FF}}};
            for (auto& x : lw) want[b + x.first] = x.second;
            for (int k : {0, 1, 5, 6, 7, 9, 11, 13, 15, 19, 20, 24, 25, 26, 27, 28, 30, 31, 32, 36, 37, 38})
                want[b + k] = {D, 1};
        }
        for (auto& kv : t) {
            auto w = want.find(kv.first);
            if (w == want.end()) continue;
            const std::vector<int64_t>& dm = kv.second.dims;
            int64_t rest = 1;
            for (size_t a = 1; a < dm.size(); ++a) rest *= dm[a];
            const int64_t lead = dm.empty() ? 1 : dm[0];
            if (lead != w->second.first || rest != w->second.second) {
                std::string s;
                for (int64_t x : dm) s += (s.empty() ? "" : " x ") + std::to_string(x);
                *err = pk_tensor_name(kv.first) + ": shape [" + s + "], expected [" + std::to_string(w->second.first) +
                       "][" + std::to_string(w->second.second) + "]";
                return false;
            }
        }
    }
    out->dims = d;
    for (auto& kv : t) out->tensors[kv.first] = std::move(kv.second.v);
    const std::string voc = dir + "/vocab.txt";
    if (file_exists(voc) && !read_vocab(voc, d.n_vocab, &out->pieces, err)) return false;
    return true;
}

}  // namespace spt
