// vocab.h -- the Whisper token vocabulary of a ggml model file: detokenisation (whisper.cpp
// whisper_token_to_str) and the greedy longest-match tokeniser whisper_full uses for
// initial_prompt (whisper.cpp whisper_tokenize / tokenize).  Spittle passes its custom-words
// ("jargon") prompt as initial_prompt (/root/reference/src-tauri/src/jargon.rs:594,
// transcription.rs:445-499), so this is on the path of every request that carries one.
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

namespace spt {

// special token ids (whisper.cpp whisper_vocab + multilingual shift)
struct Specials {
    int eot, sot, translate, transcribe, solm, prev, nosp, not_, beg, n_langs;
};
Specials specials_for(int n_vocab);
int lang_id(const std::string& code);  // whisper.cpp g_lang order; -1 if unknown
const char* lang_code(int id);         // nullptr if out of range

class Vocab {
public:
    // file_tokens: the vocabulary section of the model file (byte strings); ids from its end up
    // to n_vocab get whisper.cpp's bracketed names of the special / timestamp tokens
    Vocab(const std::vector<std::string>& file_tokens, int n_vocab, const Specials& sp);
    int size() const { return (int)id_to_tok_.size(); }
    const std::string& str(int id) const;  // "" when out of range
    int id(const std::string& tok) const;  // token_to_id; -1 when absent
    // whisper_tokenize: split with the GPT-2 pre-tokenisation pattern, then cover each piece
    // with the longest vocabulary entries from the left.  Bytes no entry covers are skipped
    // (whisper.cpp logs "unknown token" and goes on); *n_unknown counts them.
    std::vector<int> tokenize(const std::string& text, int* n_unknown) const;

private:
    std::vector<std::string> id_to_tok_;
    std::unordered_map<std::string, int> tok_to_id_;
    size_t max_len_ = 0;
};

}  // namespace spt
