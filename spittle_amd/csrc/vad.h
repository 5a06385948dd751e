// vad.h -- the capture-side voice-activity gate on the device: Silero VAD v4
// (the model file that ships with the app, resources/models/silero_vad_v4.onnx; /root/reference/
// src-tauri/src/managers/audio.rs:295-307) run over every 30 ms frame of a recorded stream, with
// the app's SmoothedVad(prefill 15, hangover 15, onset 2) on top (audio.rs:132-134,
// audio_toolkit/vad/smoothed.rs:43-104, vad/silero.rs:32-51).
//
// The network per 480-sample frame [read from the ONNX graph's 16 kHz branch]: reflect-pad 96 on
// both sides -> STFT as a stride-64 convolution with 258 basis rows of 256 taps (7 steps) -> magnitude ->
// log(1 + 2^20 mag) minus its smoothed mean (adaptive normalisation) -> [magnitude | normalised]
// 258 channels -> four depthwise-separable residual conv blocks with stride-2 1x1 convolutions
// between them (258 -> 16 -> 32 -> 32 -> 64 channels, 7 -> 4 -> 2 -> 1 steps) -> 2-layer LSTM (64; state
// carried from frame to frame) -> ReLU -> 1x1 conv -> sigmoid = speech probability.
//
// Device mapping: the convolutional front end of every frame of a stream is independent, one
// workgroup per frame (all frames at once); the LSTM recurrence is sequential, one 512-thread
// workgroup in which the two layers run one frame apart (layer 2 of frame s - 1 beside layer 1
// of frame s), each thread holding one gate row's 128 weights in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace spt {

constexpr int kVadFrame = 480;  // 30 ms at 16 kHz (vad/silero.rs:8-10)

struct SileroHost;  // the weights as read from the ONNX file (host)

class VadEngine {
public:
    VadEngine(const std::string& model_path, int device);
    ~VadEngine();
    VadEngine(const VadEngine&) = delete;
    VadEngine& operator=(const VadEngine&) = delete;

    // speech probability of each of n_frames consecutive 480-sample frames of pcm (host), the
    // LSTM state carried in from the previous call and out to the next (vad-rs keeps h, c)
    void probs(const float* pcm_host, int n_frames, float* probs_host);
    void reset_state();  // h = c = 0 (a new SileroVad)
    double last_ms() const { return last_ms_; }

private:
    void select() const;
    int dev_;
    hipStream_t st_ = nullptr;
    hipEvent_t ev_[2] = {nullptr, nullptr};
    char* wbuf_ = nullptr;     // every weight, f32, one allocation
    float* state_ = nullptr;   // h [2][64], c [2][64]
    float* pcm_ = nullptr;
    float* feat_ = nullptr;    // [frames][64]
    float* prob_ = nullptr;
    int cap_frames_ = 0;
    double last_ms_ = 0;
    struct Ptrs;
    Ptrs* p_ = nullptr;
    void ensure(int n_frames);
};

// SmoothedVad (vad/smoothed.rs): per frame, Noise or Speech(samples), the samples being the frame
// itself or, at an onset, the prefill buffer plus the frame
class SmoothedVad {
public:
    SmoothedVad(int prefill, int hangover, int onset) : prefill_(prefill), hangover_(hangover), onset_(onset) {}
    // returns 0 = Noise, 1 = Speech(frame), 2 = Speech(prefill + frame); appends the kept samples
    int push(const float* frame, int n, bool voice, std::vector<float>* out);
    // a frame the inner VAD rejects (not 480 samples): buffered, then kept as Speech(frame) by the
    // recorder's unwrap_or (recorder.rs:298), the state machine untouched
    void push_unchecked(const float* frame, int n, std::vector<float>* out);
    void reset();

private:
    int prefill_, hangover_, onset_;
    std::vector<std::vector<float>> buf_;
    int hang_ = 0, ons_ = 0;
    bool in_speech_ = false;
    void buffer(const float* frame, int n);
};

}  // namespace spt
