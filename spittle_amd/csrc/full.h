// full.h -- whisper_full's window loop over the device engine: seek-driven 30 s windows,
// temperature fallback, segments with timestamps, prompt_past conditioning.
//
// Restates whisper.cpp whisper_full_with_state (~1.7.x, vendored by whisper-rs-sys 0.11.1,
// /root/reference/src-tauri/Cargo.lock:8156-8174; not vendored here), which transcribe-rs'
// WhisperEngine::transcribe_samples calls (/root/reference/src-tauri/src/managers/
// transcription.rs:494-503) and whose segment texts it joins into TranscriptionResult.text.
// The per-token rules run on the device (k_sample.hip); this file owns what whisper.cpp does
// between decoder passes: the seek loop, decoder ranking and fallback, segment assembly.
//
// As whisper.cpp: ONE log-mel of each whole utterance (global max - 8 clamp), each window's
// encoder input = frames [seek, seek + 3000) of it, one encoder run per window shared by every
// temperature and every decoder of the utterance (Engine::load_utterances / encode_windows /
// decode).  Difference: temperature draws come from a
// counter-based stream, not mt19937.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace spt {

class Engine;
class Vocab;

struct FullParams {  // whisper_full_params
    bool no_timestamps = false;
    bool suppress_blank = true;
    bool suppress_nst = false;    // suppress_non_speech_tokens (needs a vocabulary)
    bool translate = false;
    float temperature = 0.0f;
    float temperature_inc = 0.2f;  // 0: no fallback
    int best_of = 5;               // decoders per window at temperature > 0
    int beam_size = 1;             // > 1: beam search at temperature 0 (WHISPER_SAMPLING_BEAM_SEARCH)
    float entropy_thold = 2.4f;
    float logprob_thold = -1.0f;
    float max_initial_ts = 1.0f;
    int max_tokens = 0;
    int n_max_text_ctx = 16384;
    uint64_t seed = 0;
};

struct FullSegment {
    int64_t t0, t1;   // 10 ms units (whisper_full_get_segment_t0 / t1)
    std::string text;
    int i0, n;        // its tokens in FullResult::tokens
};

struct FullResult {
    std::vector<int> tokens;        // every window's chosen decoder, result_len tokens each
    std::vector<float> plog, tid;   // per token: log-probability, timestamp id
    std::vector<FullSegment> segments;
    std::string text;               // concatenated segment texts
    int n_windows = 0;
    int n_fallbacks = 0;            // decodes repeated at a higher temperature (all windows)
    int lang_tok = -1;              // the language token decoded with (-1: English-only model)
};

// pcm[u][n[u]] host mono 16 kHz; prompt: whisper_full_params.prompt_tokens (already
// tokenised); lang_tok >= 0 fixes the language, -1 auto-detects once per utterance on its
// first window (multilingual models), ignored for English-only models
void whisper_full_batch(Engine& e, const Vocab* vocab, const std::vector<const float*>& pcm,
                        const std::vector<int>& n, const FullParams& p, const std::vector<int>& prompt, int lang_tok,
                        std::vector<FullResult>* out);

// the non-speech token ids of a vocabulary (whisper_process_logits' suppress list)
std::vector<int> non_speech_tokens(const Vocab& v);

}  // namespace spt
