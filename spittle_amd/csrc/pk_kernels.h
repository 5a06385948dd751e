// pk_kernels.h -- host launchers of the Parakeet-V3 (FastConformer-TDT) kernels (k_pk.hip).
//
// Batch layout: B utterances padded to the longest one; row (b, t) of a [B * Tp][...] tensor is
// b * Tp + t.  Per-utterance lengths live on the device (lens[b][4] = mel frames T, then the
// frame counts after each of the three stride-2 stages T1, T2, T3) and every kernel that mixes
// frames masks t >= len, so a padded batch computes each utterance exactly as alone.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spt {

constexpr int PK_NFFT = 512, PK_HOP = 160, PK_NBIN = 257, PK_DFT_N = 640;  // DFT GEMM columns (re | im | 0)

// frames[(b * Tp + t)][i] = window[i] * preemph(pcm_b)[t * 160 + i - 256] (zero outside [0, n_b))
void pk_frames(const float* pcm, int64_t stride, const int* nsamp, int B, int Tp, const float* window, float* frames,
               hipStream_t st);
// log(mel + 2^-24) of each row's power spectrum: spec [M][640] (re 0..256 | im 257..513) -> mel [M][n_mels]
void pk_melpow(const float* spec, int M, const float* fb, int n_mels, float* mel, hipStream_t st);
// per-feature normalisation over each utterance's T frames (unbiased std + 1e-5), rows >= T zeroed
void pk_mel_norm(float* mel, const int* lens, int B, int Tp, int n_mels, hipStream_t st);

// conv0: Conv2d(1, C, 3, s2, p1) + ReLU over mel [B][Tp][F] (f32) -> y [B][T1p][F1][C] (dtype)
void pk_conv0(int dtype, const float* mel, const int* lens, int B, int Tp, int F, const float* w, const float* bias,
              int C, void* y, int T1p, int F1, hipStream_t st);
// depthwise Conv2d(C, C, 3, s2, p1, groups=C): x [B][Tip][Fi][C] -> y [B][Top][Fo][C]; input
// frames >= lens[b][stage] read as zero
void pk_dwconv(int dtype, const void* x, const int* lens, int stage, int B, int Tip, int Fi, const float* w,
               const float* bias, int C, void* y, int Top, int Fo, hipStream_t st);
// relative positional encoding rows for positions Tp-1 .. -(Tp-1): pe [2Tp-1][d] (dtype)
void pk_relpos(int dtype, int Tp, int d, void* pe, hipStream_t st);
// rel-pos multi-head attention: qkv [B*Tp][3d] (q | k | v), p [2Tp-1][ldp] (layer slice of the
// projected positions), u / v biases [H][dk]; keys >= T3_b masked; out [B*Tp][d]
void pk_rel_attn(int dtype, const void* qkv, const void* p, int ldp, const float* pu, const float* pv,
                 const int* lens, int B, int Tp, int H, int dk, void* out, hipStream_t st);
// conformer convolution module after pw1: a [B*Tp][2d] -> GLU -> depthwise K taps (frames
// outside [0, T3_b) zero) -> BatchNorm (eval) -> Swish -> out [B*Tp][d]
void pk_conv_module(int dtype, const void* a, const int* lens, int B, int Tp, int d, int K, const float* dw_w,
                    const float* dw_b, const float* bn_g, const float* bn_b, const float* bn_m, const float* bn_v,
                    void* out, hipStream_t st);

// weight placement (f32 source on the device -> engine storage)
enum { PK_PLACE_COPY = 0, PK_PLACE_TRANSPOSE = 1, PK_PLACE_SUBPERM = 2 };
// COPY: dst[i] = src[i] (dtype); TRANSPOSE: src [N][K] -> f32 dst[(row0 + k) * ld + n];
// SUBPERM: src [N][C * F] (channel-major flatten) -> dst [N][F * C] (dtype)
void pk_place(int mode, int dtype, const float* src, int N, int K, void* dst, int ld, int row0, int C, int F,
              hipStream_t st);

// ---- TDT greedy decoding (f32 prediction network + joint)
struct PkState {         // per row, device
    int t, at_t, n_out, done, upd, tok;
};
enum { PKX_LSTM0 = 0, PKX_LSTM1 = 1, PKX_PRED = 2, PKX_JOINT = 3 };
struct PkGemvArgs {
    const float* WT; int Npad, K;  // W^T [K][Npad]
    int ksplit;                    // K / ksplit rows per split (split s -> part[s])
    float* part;                   // [ksplit][B][Npad]
    int B, P;
    const PkState* st;
    const float* emb;              // PKX_LSTM0: [V+1][P]
    const float* h0; const float* h1;  // [B][P]
    const float* fe; int T3p;      // PKX_JOINT: encoder projection [B*T3p][P]
    const float* pred_part; int pred_split, pred_Npad; const float* pred_b;  // PKX_JOINT: gp = sum + b (upd rows)
    float* gp;                     // [B][P] stored prediction projection
};
void pk_gemv(int xmode, const PkGemvArgs& a, hipStream_t s);
// LSTM cell of the rows with upd: gates = sum of part slabs + b_ih + b_hh (i, f, g, o)
void pk_lstm_cell(const float* part, int ksplit, int Npad, const float* b_ih, const float* b_hh, int B, int P,
                  const PkState* st, float* h, float* c, hipStream_t s);
struct PkFinArgs {
    const float* part; int ksplit, Npad;  // joint slabs
    const float* bias;                    // [V + 1 + n_dur]
    int V, n_dur, max_symbols, B, cap;
    const int* lens;                      // T3 per row at lens[b * 4 + 3]
    PkState* st;
    int* out_tok; int* out_frame; float* out_t1; float* out_t2;  // [B][cap]
};
void pk_joint_fin(const PkFinArgs& a, hipStream_t s);
// rows start at t = 0 with the blank symbol pending (upd, tok = V); h / c: n floats zeroed
void pk_state_init(PkState* st, int B, int V, float* h, float* c, int n, hipStream_t s);

}  // namespace spt
