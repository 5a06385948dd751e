// ggml_file.h -- reader of whisper.cpp's legacy ggml model files (the .bin files Spittle's
// model catalog ships: /root/reference/src-tauri/resources/model_catalog.json, resolved by
// ModelManager::get_model_path, /root/reference/src-tauri/src/managers/model.rs:804-847).
//
// Layout (whisper.cpp whisper_model_load): magic 0x67676d6c "ggml"; 11 int32 hparams (n_vocab,
// n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer, n_text_ctx, n_text_state,
// n_text_head, n_text_layer, n_mels, ftype); the mel filterbank (int32 n_mel, int32 n_fft,
// n_mel * n_fft f32); the vocabulary (int32 n, then n x {uint32 len, bytes}); then tensors to
// the end of the file: int32 n_dims, int32 name_len, int32 ggml type, int32 ne[n_dims], the
// name, the data (ggml row-major: ne[0] fastest; no padding).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace spt {

struct GgmlTensor {
    std::string name;
    int type = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    int n_dims = 0;
    const uint8_t* data = nullptr;  // into the mapping
    size_t nbytes = 0;
    int64_t numel() const { return ne[0] * ne[1] * ne[2] * ne[3]; }
};

struct GgmlHparams {
    int n_vocab, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int n_text_ctx, n_text_state, n_text_head, n_text_layer, n_mels, ftype;
};

class GgmlFile {
public:
    ~GgmlFile();
    // false + *err on any format violation (truncation, unknown type, bad sizes)
    bool open(const std::string& path, std::string* err);
    const GgmlHparams& hparams() const { return hp_; }
    int n_mel_filters() const { return n_mel_; }
    int n_fft() const { return n_fft_; }
    const std::vector<float>& mel_filters() const { return filters_; }  // [n_mel][n_fft]
    const std::vector<std::string>& vocab() const { return vocab_; }
    const GgmlTensor* find(const std::string& name) const;
    size_t n_tensors() const { return tensors_.size(); }

    // block geometry of a ggml type: elements per block, bytes per block (0 if unsupported)
    static void type_block(int type, int* blck, int* bytes);

private:
    GgmlHparams hp_{};
    int n_mel_ = 0, n_fft_ = 0;
    std::vector<float> filters_;
    std::vector<std::string> vocab_;
    std::vector<GgmlTensor> tensors_;
    std::map<std::string, size_t> index_;
    void* map_ = nullptr;
    size_t size_ = 0;
};

// host reference dequantisation of n elements (a multiple of the type's block) to f32
bool ggml_dequant_host(int type, const uint8_t* src, int64_t n, float* dst);

}  // namespace spt
