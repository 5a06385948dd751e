// vocab.cpp -- see vocab.h.
#include "vocab.h"

#include <algorithm>
#include <regex>

namespace spt {

Specials specials_for(int n_vocab) {
    // whisper.cpp whisper_vocab defaults, shifted for multilingual vocabularies in
    // whisper_model_load (language count = n_vocab - 51765 - multilingual)
    Specials s{50256, 50257, 50357, 50358, 50359, 50360, 50361, 50362, 50363, 0};
    const bool multi = n_vocab >= 51865;
    const int n_langs = n_vocab - 51765 - (multi ? 1 : 0);
    if (multi) {
        s.eot++;
        s.sot++;
        const int dt = n_langs - 98;
        s.translate += dt; s.transcribe += dt; s.solm += dt; s.prev += dt; s.nosp += dt; s.not_ += dt; s.beg += dt;
        s.n_langs = n_langs;
    }
    return s;
}

static const char* const kLangs[] = {
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
    "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
    "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
    "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
    "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
    "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue"};
constexpr int kNumLangs = (int)(sizeof(kLangs) / sizeof(kLangs[0]));

int lang_id(const std::string& code) {
    for (int i = 0; i < kNumLangs; ++i)
        if (code == kLangs[i]) return i;
    return -1;
}

const char* lang_code(int id) { return (id >= 0 && id < kNumLangs) ? kLangs[id] : nullptr; }


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
