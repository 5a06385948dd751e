// onnx_fuzz.cpp -- the host code that reads the app's downloaded / shipped ONNX files, built
// standalone with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_host_sanitizers.py:
// the protobuf reader (onnx_pb.cpp), the Parakeet model-directory mapper (pk_onnx.cpp) and the
// Silero VAD graph walk + device-blob packing (vad_model.cpp).  No device code.
//   onnx_fuzz parakeet <dir>   load_parakeet_onnx(dir): dims, tensors, vocabulary
//   onnx_fuzz vad <file.onnx>  load_silero(file) + silero_blob
// Prints "parsed: ..." or "rejected: <reason>"; exit status 0 either way.
#include <stdio.h>
#include <string.h>

#include <string>

#include "../../spittle_amd/csrc/pk_onnx.h"
#include "../../spittle_amd/csrc/vad_model.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    std::string err;
    if (!strcmp(argv[1], "parakeet")) {
        spt::PkOnnxModel m;
        if (!spt::load_parakeet_onnx(argv[2], &m, &err)) {
            printf("rejected: %s\n", err.c_str());
            return 0;
        }
        double sum = 0.0;
        size_t n = 0;
        for (auto& kv : m.tensors) {
            n += kv.second.size();
            for (float v : kv.second) sum += v;
        }
        printf("parsed: %zu tensors, %zu values (sum %.6g), d %d, layers %d, %zu pieces, %d quantised\n",
               m.tensors.size(), n, sum, m.dims.d, m.dims.n_layers, m.pieces.size(), m.n_quantized);
        return 0;
    }
    if (!strcmp(argv[1], "vad")) {
        spt::SileroHost m;
        if (!spt::load_silero(argv[2], &m, &err)) {
            printf("rejected: %s\n", err.c_str());
            return 0;
        }
        spt::SileroOff o;
        const std::vector<float> blob = spt::silero_blob(m, &o);
        double sum = 0.0;
        for (float v : blob) sum += v;
        printf("parsed: blob %zu floats (sum %.6g), mag_scale %g\n", blob.size(), sum, m.mag_scale);
        return 0;
    }
    return 2;
}
