// onnx_pb.h -- a minimal, copy-free reader of ONNX model files (protobuf wire format), enough to
// take the initializers and the node graph out of the Parakeet-V3 export the app downloads
// (parakeet-tdt-0.6b-v3-int8: encoder-model.int8.onnx, decoder_joint-model.int8.onnx;
// /root/reference/src-tauri/resources/model_catalog.json:229-241).  No protobuf library: the
// file is memory-mapped and the few message types ONNX needs (ModelProto -> GraphProto ->
// NodeProto / TensorProto / AttributeProto, onnx.proto field numbers) are decoded by hand.
// Nothing in the file is executed; malformed input is rejected with an error, never trusted
// (every length is bounded against the mapping).
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace spt {
namespace onnx {

enum DataType { T_FLOAT = 1, T_UINT8 = 2, T_INT8 = 3, T_INT32 = 6, T_INT64 = 7, T_FLOAT16 = 10, T_DOUBLE = 11,
                T_BFLOAT16 = 16 };

struct Tensor {
    std::string name;
    std::vector<int64_t> dims;
    int data_type = 0;
    const uint8_t* raw = nullptr;  // raw_data inside the mapping (or external data), else null
    size_t raw_len = 0;
    std::vector<float> f32;        // float_data (packed or not)
    std::vector<int64_t> i64;      // int32_data / int64_data (int8, uint8, fp16 bits travel here too)
    std::string ext_location;      // external data (data_location = EXTERNAL)
    int64_t ext_offset = 0, ext_length = -1;
    int64_t numel() const;
    // the values as f32 (FLOAT, FLOAT16, BFLOAT16, DOUBLE, INT8, UINT8, INT32, INT64); false + err otherwise
    bool to_f32(std::vector<float>* out, std::string* err) const;
};

struct Graph;
struct Attribute {
    std::string name;
    int64_t i = 0;
    float f = 0.f;
    std::string s;
    std::vector<int64_t> ints;
    std::shared_ptr<Graph> g;  // subgraph (If / Loop branches)
};

struct Node {
    std::string name, op_type, domain;
    std::vector<std::string> inputs, outputs;
    std::vector<Attribute> attrs;
    const Attribute* attr(const std::string& n) const;
};

struct Graph {
    std::vector<Node> nodes;
    std::vector<Tensor> initializers;
    std::vector<std::string> outputs;
    const Tensor* find(const std::string& name) const {
        for (const Tensor& t : initializers)
            if (t.name == name) return &t;
        return nullptr;
    }
};

class Model {
public:
    // maps and parses path; external data files are resolved next to it
    bool open(const std::string& path, std::string* err);
    const Graph& graph() const { return graph_; }
    ~Model();

private:
    bool resolve_external(std::string* err);
    std::string path_;
    const uint8_t* map_ = nullptr;
    size_t len_ = 0;
    std::vector<std::pair<const uint8_t*, size_t>> ext_maps_;
    Graph graph_;
};

}  // namespace onnx
}  // namespace spt
