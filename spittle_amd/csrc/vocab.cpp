// vocab.cpp -- see vocab.h.
#include "vocab.h"

#include <regex>

#include "engine.h"

namespace spt {

Vocab::Vocab(const std::vector<std::string>& file_tokens, int n_vocab, const Specials& sp) {
    const int n = std::max<int>(n_vocab, (int)file_tokens.size());
    id_to_tok_.resize(n);
    for (int i = 0; i < n; ++i) {
        std::string w;
        if (i < (int)file_tokens.size()) w = file_tokens[i];
        else if (i > sp.beg) w = "[_TT_" + std::to_string(i - sp.beg) + "]";
        else if (i == sp.eot) w = "[_EOT_]";
        else if (i == sp.sot) w = "[_SOT_]";
        else if (i == sp.translate) w = "[_TRANSLATE_]";
        else if (i == sp.transcribe) w = "[_TRANSCRIBE_]";
        else if (i == sp.solm) w = "[_SOLM_]";
        else if (i == sp.prev) w = "[_PREV_]";
        else if (i == sp.nosp) w = "[_NOSP_]";
        else if (i == sp.not_) w = "[_NOT_]";
        else if (i == sp.beg) w = "[_BEG_]";
        else if (i > sp.sot && i <= sp.sot + sp.n_langs) w = std::string("[_LANG_") + lang_code(i - sp.sot - 1) + "]";
        else w = "[_extra_token_" + std::to_string(i) + "]";
        id_to_tok_[i] = w;
        tok_to_id_[w] = i;  // a later duplicate wins, as in whisper_model_load
        max_len_ = std::max(max_len_, w.size());
    }
}

const std::string& Vocab::str(int id) const {
    static const std::string empty;
    return (id >= 0 && id < (int)id_to_tok_.size()) ? id_to_tok_[id] : empty;
}

int Vocab::id(const std::string& tok) const {
    auto it = tok_to_id_.find(tok);
    return it == tok_to_id_.end() ? -1 : it->second;
}

std::vector<int> Vocab::tokenize(const std::string& text, int* n_unknown) const {
    // GPT-2's pre-tokenisation pattern as whisper.cpp states it for std::regex (ECMAScript,
    // "C" locale classes: bytes >= 0x80 are neither alpha nor digit nor space)
    static const std::regex re(R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
    std::vector<std::string> words;
    std::string rest = text;
    std::smatch m;
    while (std::regex_search(rest, m, re)) {
        for (const auto& sub : m) words.push_back(sub);
        rest = m.suffix();
    }
    std::vector<int> out;
    int unknown = 0;
    for (const std::string& w : words) {
        const int n = (int)w.size();
        int i = 0;
        while (i < n) {
            bool found = false;
            for (int j = std::min<int>(n, i + (int)max_len_); j > i; --j) {
                auto it = tok_to_id_.find(w.substr(i, j - i));
                if (it != tok_to_id_.end()) {
                    out.push_back(it->second);
                    i = j;
                    found = true;
                    break;
                }
            }
            if (!found) {
                ++unknown;
                ++i;
            }
        }
    }
    if (n_unknown) *n_unknown = unknown;
    return out;
}

}  // namespace spt
