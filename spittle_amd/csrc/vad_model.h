// vad_model.h -- the Silero VAD v4 weights read from the app's ONNX file (host only; see vad.h for
// the network).  Separate from vad.hip so the parser of this untrusted file builds and runs under
// AddressSanitizer / UBSan without a device (tests/native/host_fuzz.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace spt {

constexpr int kPadL = 96;  // reflect padding of the frame on both sides (the graph's Pad)
constexpr int kNBlk = 15;  // encoder convolutions (graph order, vad_model.cpp kBlk)

struct ConvW {  // one Conv node: weight [out][in / group][k], bias [out]
    int out = 0, in_g = 0, k = 0, group = 1, stride = 1, pad = 0;
    std::vector<float> w, b;
};
struct SileroHost {
    ConvW stft, filt;                 // forward basis (258 x 256, stride 64), adaptive-normalisation filter (7)
    ConvW blk[17];                    // the encoder's convolutions in graph order
    ConvW dec;                        // decoder 1x1 conv 64 -> 1
    std::vector<float> lw[2], lr[2], lb[2];  // LSTM layers: W [256][64], R [256][64], B [512] (ONNX gates i, o, f, c)
    float pad_left = 96.f, pad_right = 96.f, mag_scale = 1048576.f;
};

// the 16 kHz branch of the graph's top-level If (sr == 16000): its Conv nodes in graph order and the
// two LSTM nodes of the branch that takes the caller's state; false + *err if the file is not that
bool load_silero(const std::string& path, SileroHost* m, std::string* err);

// the device blob: every tensor f32 at these float offsets (64-aligned)
struct SileroOff {
    int64_t stft_w, filt_w, blk_w[kNBlk], blk_b[kNBlk], dec_w, dec_b, lw[2], lr[2], lb[2], total;
};
// pack a loaded model into one blob (LSTM biases summed: b_ih + b_hh)
std::vector<float> silero_blob(const SileroHost& m, SileroOff* o);

}  // namespace spt
