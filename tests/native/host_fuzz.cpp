// host_fuzz.cpp -- the host-only parts of the library that read untrusted input (the ggml model
// file parser, the tokenizer, the block dequantisers), built standalone with AddressSanitizer and
// UndefinedBehaviorSanitizer by tests/test_host_sanitizers.py.
//   host_fuzz <model.bin> <text>   open the file; if it parses, tokenize the text with its
//                                  vocabulary and dequantise every tensor on the host
// Exit status 0 when every step either succeeded or reported a clean error.
#include <stdio.h>

#include <string>
#include <vector>

#include "../../spittle_amd/csrc/ggml_file.h"
#include "../../spittle_amd/csrc/vocab.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    spt::GgmlFile f;
    std::string err;
    if (!f.open(argv[1], &err)) {
        printf("rejected: %s\n", err.c_str());
        return 0;
    }
    spt::Vocab v(f.vocab(), f.hparams().n_vocab, spt::specials_for(f.hparams().n_vocab));
    int unk = 0;
    const std::vector<int> t = v.tokenize(argv[2], &unk);
    size_t n_bytes = 0;
    for (int id : t) n_bytes += v.str(id).size();
    const char* names[] = {"t0", "t1", "t2", "t3", "t4", "t5", "t6", "t7"};
    size_t n_deq = 0;
    for (const char* nm : names) {
        const spt::GgmlTensor* g = f.find(nm);
        if (!g) continue;
        std::vector<float> out((size_t)g->numel());
        if (spt::ggml_dequant_host(g->type, g->data, g->numel(), out.data())) n_deq++;
    }
    printf("parsed: %zu tensors, %zu tokens (%zu bytes, %d unknown), %zu dequantised\n", f.n_tensors(), t.size(),
           n_bytes, unk, n_deq);
    return 0;
}
