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
enum { PK_PLACE_COPY = 0, PK_PLACE_TRANSPOSE = 1, PK_PLACE_SUBPERM = 2, PK_PLACE_LSTM = 3, PK_PLACE_BLOCKED = 4 };
// COPY: dst[i] = src[i] (dtype); TRANSPOSE: src [N][K] -> f32 dst[(row0 + k) * ld + n];
// SUBPERM: src [N][C * F] (channel-major flatten) -> dst [N][F * C] (dtype)
void pk_place(int mode, int dtype, const float* src, int N, int K, void* dst, int ld, int row0, int C, int F,
              hipStream_t st);

// ---- TDT greedy decoding (f32 prediction network + joint)
struct PkState {         // per row, device
    int t, at_t, n_out, done, upd, tok;
    int t3p;  // this call's frame stride of fe (set by pk_state_init, so a captured step is shape-free)
};
// One decode step = LSTM layer 0, LSTM layer 1, prediction projection, joint, fin.  The LSTM
// states ping-pong between two buffers per layer (a stage's workgroups read every unit of the
// previous state while writing their own units of the next).
enum { PKD_LSTM = 0, PKD_PRED = 1, PKD_JOINT = 2 };
struct PkDecArgs {
    const float* WT; int ld, K, N;  // blocked W^T [ld / DO][K][DO] (pk_place_lstm / pk_place_blocked); ld = padded N
    const float* b0; const float* b1;  // LSTM: b_ih, b_hh; PRED / JOINT: bias
    int B, P, V, n_dur;
    const PkState* st;
    const float* xin;               // LSTM: input rows [B][P] (layer 0: the token embeddings); PRED: h1

    const float* h_in; const float* c_in; float* h_out; float* c_out;  // LSTM state [B][P]
    const float* fe;                // JOINT: each row's current-frame encoder projection [B][P]
    float* gp;                      // PRED: out (rows with upd); JOINT: in [B][P]
    float4* part; int n_tiles;      // JOINT: per-workgroup top-2 {v1, i1, v2, -} [B][n_tiles]
    float* dur;                     // JOINT: duration logits [B][n_dur]
};
void pk_decode_stage(int mode, const PkDecArgs& a, hipStream_t s);
// one-time kernel attributes (before any stream capture)
void pk_prepare();
// outputs per workgroup of the joint stage (its top-2 partials per row: ld / pk_joint_tile())
int pk_joint_tile();
struct PkFinArgs {
    const float4* part; int n_tiles;
    const float* dur;
    int V, n_dur, max_symbols, B, cap;
    const int* lens;                      // T3 per row at lens[b * 4 + 3]
    PkState* st;
    int P;
    const float* emb; const float* fe;    // embedding [V+1][P]; encoder projection [B*T3p][P]
    float* xemb; float* fecur;            // out: next step's LSTM-0 input / current-frame row [B][P]
    int* out_tok; int* out_frame; float* out_t1; float* out_t2;  // [B][cap]
};
void pk_joint_fin(const PkFinArgs& a, hipStream_t s);
// rows start at t = 0 with the blank symbol pending (upd, tok = V); h / c: n floats zeroed; xemb
// zero (the blank row), fecur = frame 0 of fe [B*T3p][P]
void pk_state_init(PkState* st, int B, int V, float* h, float* c, int n, float* xemb, float* fecur, const float* fe,
                   const int* lens,
                   int T3p, int P, hipStream_t s);
// LSTM weight [4P][P] (gate rows i, f, g, o) -> rows row0.. of the blocked, gate-interleaved W^T
// [P / 4][2P][16]
void pk_place_lstm(const float* src, int P, float* dst, int row0, hipStream_t s);
// W [N][K] -> the blocked W^T [ceil(N / DO)][K][DO] of the PKD_PRED / PKD_JOINT stage
void pk_place_blocked(const float* src, int N, int K, int mode, float* dst, hipStream_t s);

}  // namespace spt
