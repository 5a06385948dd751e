// pk_onnx.h -- the Parakeet-V3 model directory the app downloads and hands to
// ParakeetEngine::load_model_with_params(&path, ParakeetModelParams::int8())
// (/root/reference/src-tauri/src/managers/transcription.rs:278-297; catalog entry
// parakeet-tdt-0.6b-v3-int8, /root/reference/src-tauri/resources/model_catalog.json:229-241):
// the onnx-asr export of NeMo's parakeet-tdt-0.6b-v3 that transcribe-rs 0.2.3 reads
// [upstream, recalled]: encoder-model[.int8].onnx, decoder_joint-model[.int8].onnx,
// nemo128.onnx (the preprocessor; not read: the log-mel is this library's own k_pk.hip), vocab.txt.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "parakeet.h"

namespace spt {

struct PkOnnxModel {
    PkDims dims;
    std::map<int, std::vector<float>> tensors;  // engine tensor id -> f32 values in NeMo's layout
    std::vector<std::string> pieces;            // vocab.txt: token id -> piece (blank excluded)
    std::string encoder_file, decoder_file;
    int n_quantized = 0;                        // initializers dequantized (int8 / uint8 + scale + zero point)
};

// the NeMo state-dict name of an engine tensor id (error messages)
std::string pk_tensor_name(int tid);

// true: `path` is a directory holding an encoder-model*.onnx (the app's model directory)
bool is_parakeet_onnx_dir(const std::string& path);

// parse both graphs, dequantise, map every initializer onto the engine's tensor table and infer
// the model's dimensions; false + err on anything missing or inconsistent
bool load_parakeet_onnx(const std::string& dir, PkOnnxModel* out, std::string* err);

}  // namespace spt
