// vad_model.cpp -- see vad_model.h.  Reads the graph with the ONNX protobuf reader (onnx_pb.cpp).
#include "vad_model.h"

#include <algorithm>

#include "onnx_pb.h"

namespace spt {

namespace {

const onnx::Tensor* find_t(const std::vector<const onnx::Graph*>& scopes, const std::string& name) {
    for (auto it = scopes.rbegin(); it != scopes.rend(); ++it)
        if (const onnx::Tensor* t = (*it)->find(name)) return t;
    return nullptr;
}

std::vector<float> vals(const std::vector<const onnx::Graph*>& scopes, const std::string& name, std::string* err) {
    const onnx::Tensor* t = find_t(scopes, name);
    std::vector<float> v;
    if (!t) { *err = "Silero model: no initializer '" + name + "'"; return v; }
    if (!t->to_f32(&v, err)) v.clear();
    return v;
}

bool read_conv(const onnx::Node& n, const std::vector<const onnx::Graph*>& sc, ConvW* c, std::string* err) {
    const onnx::Tensor* w = n.inputs.size() > 1 ? find_t(sc, n.inputs[1]) : nullptr;
    if (!w || w->dims.size() != 3) { *err = "Silero model: Conv '" + n.name + "' weight is not a 1-D conv initializer"; return false; }
    c->out = (int)w->dims[0]; c->in_g = (int)w->dims[1]; c->k = (int)w->dims[2];
    if (const onnx::Attribute* a = n.attr("group")) c->group = (int)a->i;
    if (const onnx::Attribute* a = n.attr("strides"); a && !a->ints.empty()) c->stride = (int)a->ints[0];
    if (const onnx::Attribute* a = n.attr("pads"); a && !a->ints.empty()) c->pad = (int)a->ints[0];
    if (c->out < 1 || c->in_g < 1 || c->k < 1 || c->out > 4096 || c->in_g > 4096 || c->k > 4096) {
        *err = "Silero model: Conv '" + n.name + "' weight has an unexpected shape";
        return false;
    }
    if (!w->to_f32(&c->w, err)) return false;
    if (n.inputs.size() > 2 && !n.inputs[2].empty()) {
        c->b = vals(sc, n.inputs[2], err);
        if (c->b.empty()) return false;
    } else c->b.assign(c->out, 0.f);
    return (int)c->b.size() == c->out;
}

const onnx::Graph* branch(const onnx::Node& n, const char* which) {
    const onnx::Attribute* a = n.attr(which);
    return a ? a->g.get() : nullptr;
}

// expected encoder conv shapes (out, in/group, k, group, stride) in graph order
struct Shape { int out, in_g, k, group, stride; };
const Shape kBlk[17] = {
    {258, 1, 5, 258, 1}, {16, 258, 1, 1, 1}, {16, 258, 1, 1, 1},   // first_layer: dw, pw, proj
    {16, 16, 1, 1, 2},                                              // stride-2 1x1
    {16, 1, 5, 16, 1}, {32, 16, 1, 1, 1}, {32, 16, 1, 1, 1},       // encoder.3: dw, pw, proj
    {32, 32, 1, 1, 2},
    {32, 1, 5, 32, 1}, {32, 32, 1, 1, 1},                           // encoder.7: dw, pw (identity residual)
    {32, 32, 1, 1, 2},
    {32, 1, 5, 32, 1}, {64, 32, 1, 1, 1}, {64, 32, 1, 1, 1},       // encoder.11: dw, pw, proj
    {64, 64, 1, 1, 1},                                              // 1x1 before the LSTM
    {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}};

}  // namespace

bool load_silero(const std::string& path, SileroHost* m, std::string* err) {
    onnx::Model model;
    if (!model.open(path, err)) return false;
    const onnx::Graph& top = model.graph();
    // the top-level If on sr == 16000: its then branch is the 16 kHz model
    const onnx::Graph* g16 = nullptr;
    for (const onnx::Node& n : top.nodes)
        if (n.op_type == "If") g16 = branch(n, "then_branch");
    if (!g16) { *err = path + ": not the Silero VAD graph (no sample-rate If)"; return false; }
    std::vector<const onnx::Graph*> sc{&top, g16};
    std::vector<const onnx::Node*> convs;
    const onnx::Node* lstm_if = nullptr;
    for (const onnx::Node& n : g16->nodes) {
        if (n.op_type == "Conv") convs.push_back(&n);
        if (n.op_type == "If")
            if (const onnx::Graph* t = branch(n, "then_branch"))
                for (const onnx::Node& x : t->nodes)
                    if (x.op_type == "LSTM") lstm_if = &n;
        if (n.op_type == "Pad" && n.inputs.size() > 1) {
            std::vector<float> p = vals(sc, n.inputs[1], err);
            if (p.size() >= 2 && p.size() % 2 == 0) {  // [begins..., ends...]: the time (last) axis
                m->pad_left = p[p.size() / 2 - 1];
                m->pad_right = p[p.size() - 1];
            }
        }
        if (n.op_type == "Mul")
            for (const std::string& in : n.inputs)
                if (const onnx::Tensor* t = find_t(sc, in); t && t->numel() == 1) {
                    std::vector<float> v;
                    if (t->to_f32(&v, err) && v.size() == 1) m->mag_scale = v[0];
                }
    }
    // graph order: STFT basis, normalisation filter, 15 encoder convs, decoder conv
    if (convs.size() != (size_t)(2 + kNBlk + 1)) {
        *err = path + ": expected " + std::to_string(2 + kNBlk + 1) + " Conv nodes in the 16 kHz branch, found " +
               std::to_string(convs.size());
        return false;
    }
    if (!read_conv(*convs[0], sc, &m->stft, err) || !read_conv(*convs[1], sc, &m->filt, err) ||
        !read_conv(*convs.back(), sc, &m->dec, err))
        return false;
    // every shape the device blob and kernels assume (a smaller tensor would be read past its end,
    // a larger one written past its slot)
    if (m->stft.out != 258 || m->stft.in_g != 1 || m->stft.k != 256 || m->stft.stride != 64 || m->filt.out != 1 ||
        m->filt.in_g != 1 || m->filt.k != 7 || m->dec.out != 1 || m->dec.in_g != 64 || m->dec.k != 1) {
        *err = path + ": unexpected STFT / filter / decoder shapes";
        return false;
    }
    for (int i = 0; i < kNBlk; ++i) {
        if (!read_conv(*convs[2 + i], sc, &m->blk[i], err)) return false;
        const ConvW& c = m->blk[i];
        const Shape& s = kBlk[i];
        if (c.out != s.out || c.in_g != s.in_g || c.k != s.k || c.group != s.group || c.stride != s.stride ||
            (c.k == 5 && c.pad != 2)) {
            *err = path + ": encoder conv " + std::to_string(i) + " has an unexpected shape";
            return false;
        }
    }
    if (!lstm_if) { *err = path + ": no LSTM in the 16 kHz branch"; return false; }
    const onnx::Graph* with_state = branch(*lstm_if, "then_branch");  // the caller's h / c
    std::vector<const onnx::Graph*> sc2{&top, g16, with_state};
    int layer = 0;
    for (const onnx::Node& x : with_state->nodes) {
        if (x.op_type != "LSTM" || layer >= 2) continue;
        if (x.inputs.size() < 4) { *err = path + ": LSTM without bias"; return false; }
        m->lw[layer] = vals(sc2, x.inputs[1], err);
        m->lr[layer] = vals(sc2, x.inputs[2], err);
        m->lb[layer] = vals(sc2, x.inputs[3], err);
        if (m->lw[layer].size() != 256 * 64 || m->lr[layer].size() != 256 * 64 || m->lb[layer].size() != 512) {
            *err = path + ": LSTM layer " + std::to_string(layer) + " is not 64 units over 64 inputs";
            return false;
        }
        ++layer;
    }
    if (layer != 2) { *err = path + ": expected two LSTM layers"; return false; }
    if (m->pad_left != (float)kPadL || m->pad_right != (float)kPadL) { *err = path + ": unexpected STFT padding"; return false; }
    return true;
}


std::vector<float> silero_blob(const SileroHost& m, SileroOff* o) {
    *o = SileroOff{};
    int64_t p = 0;
    auto take = [&](int64_t n) { const int64_t r = p; p += (n + 63) / 64 * 64; return r; };
    o->stft_w = take(258 * 256);
    o->filt_w = take(7);
    for (int i = 0; i < kNBlk; ++i) {
        o->blk_w[i] = take((int64_t)m.blk[i].w.size());
        o->blk_b[i] = take(m.blk[i].out);
    }
    o->dec_w = take(64);
    o->dec_b = take(1);
    for (int l = 0; l < 2; ++l) { o->lw[l] = take(256 * 64); o->lr[l] = take(256 * 64); o->lb[l] = take(256); }
    o->total = p;
    std::vector<float> blob((size_t)p, 0.f);
    // each tensor into its slot, never past it (load_silero checked the shapes; this is the guard)
    auto put = [&](int64_t off, int64_t cap, const std::vector<float>& v) {
        std::copy(v.begin(), v.begin() + std::min<int64_t>(cap, (int64_t)v.size()), blob.begin() + off);
    };
    put(o->stft_w, 258 * 256, m.stft.w);
    put(o->filt_w, 7, m.filt.w);
    for (int i = 0; i < kNBlk; ++i) {
        put(o->blk_w[i], (int64_t)m.blk[i].w.size(), m.blk[i].w);
        put(o->blk_b[i], m.blk[i].out, m.blk[i].b);
    }
    put(o->dec_w, 64, m.dec.w);
    put(o->dec_b, 1, m.dec.b);
    for (int l = 0; l < 2; ++l) {
        put(o->lw[l], 256 * 64, m.lw[l]);
        put(o->lr[l], 256 * 64, m.lr[l]);
        std::vector<float> b(256, 0.f);
        if (m.lb[l].size() >= 512)
            for (int i = 0; i < 256; ++i) b[i] = m.lb[l][i] + m.lb[l][256 + i];
        put(o->lb[l], 256, b);
    }
    return blob;
}

}  // namespace spt
