// capi_vad.cpp -- the spt_vad_* half of include/spittle_hip.h (ABI 8): the recorder's voice-
// activity gate.  In the reference the recorder's consumer thread calls, per 30 ms frame from the
// FrameResampler, SmoothedVad::push_frame (SmoothedVad(SileroVad(silero_vad_v4.onnx, 0.3), 15, 15,
// 2): /root/reference/src-tauri/src/managers/audio.rs:132-134) and appends Speech frames to the
// recording (audio_toolkit/audio/recorder.rs:284-301); Cmd::Start calls vad.reset() (:343-349),
// which resets the smoothing only -- SileroVad has no reset, so its LSTM state carries over.
#include <hip/hip_runtime.h>
#include <string.h>

#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/spittle_hip.h"
#include "common.h"
#include "vad.h"

struct spt_vad {
    std::unique_ptr<spt::VadEngine> eng;
    std::unique_ptr<spt::SmoothedVad> smooth;
    float threshold = 0.3f;
    std::string err;
};

namespace {

void set_err(char* err, size_t errlen, const std::string& m) {
    if (err && errlen) {
        strncpy(err, m.c_str(), errlen - 1);
        err[errlen - 1] = 0;
    }
}

spt_status fail(spt_vad* v, spt_status s, const std::string& m) {
    if (v) v->err = m;
    return s;
}

spt_status classify(const std::exception& e) {
    if (dynamic_cast<const spt::HipError*>(&e)) return SPT_ERR_DEVICE;
    if (dynamic_cast<const std::bad_alloc*>(&e)) return SPT_ERR_OOM;
    return SPT_ERR_INTERNAL;
}

}  // namespace

extern "C" {

void spt_vad_default_params(spt_vad_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->threshold = 0.3f;        // SileroVad::new(vad_path, 0.3)
    p->prefill_frames = 15;     // SmoothedVad::new(.., 15, 15, 2)
    p->hangover_frames = 15;
    p->onset_frames = 2;
}

spt_status spt_vad_create(const char* model_path, const spt_vad_params* params, spt_vad** out, char* err,
                          size_t errlen) {
    if (!model_path || !out) {
        set_err(err, errlen, "null argument");
        return SPT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    spt_vad_params p;
    spt_vad_default_params(&p);
    if (params) p = *params;
    if (!(p.threshold >= 0.0f && p.threshold <= 1.0f)) {  // silero.rs:22-24
        set_err(err, errlen, "threshold must be between 0.0 and 1.0");
        return SPT_ERR_INVALID_ARG;
    }
    if (p.prefill_frames < 0 || p.hangover_frames < 0 || p.onset_frames < 0 || p.prefill_frames > 10000) {
        set_err(err, errlen, "frame counts must be non-negative");
        return SPT_ERR_INVALID_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_err(err, errlen, "no HIP device available");
        return SPT_ERR_DEVICE;
    }
    if (p.device < 0 || p.device >= ndev) {
        set_err(err, errlen, "device ordinal out of range");
        return SPT_ERR_INVALID_ARG;
    }
    std::unique_ptr<spt_vad> v(new (std::nothrow) spt_vad());
    if (!v) return SPT_ERR_OOM;
    try {
        v->eng.reset(new spt::VadEngine(model_path, p.device));
    } catch (const std::exception& e) {
        set_err(err, errlen, std::string("Failed to create VAD: ") + e.what());
        const spt_status s = classify(e);
        return s == SPT_ERR_INTERNAL ? SPT_ERR_LOAD : s;
    }
    v->smooth.reset(new spt::SmoothedVad(p.prefill_frames, p.hangover_frames, p.onset_frames));
    v->threshold = p.threshold;
    *out = v.release();
    return SPT_OK;
}

spt_status spt_vad_push(spt_vad* v, const float* pcm, size_t n, spt_vad_result** out) {
    if (!v || !out || (n && !pcm)) return fail(v, SPT_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    const size_t nf = n / spt::kVadFrame, rem = n % spt::kVadFrame;
    if (nf > (size_t)INT32_MAX / spt::kVadFrame) return fail(v, SPT_ERR_INVALID_ARG, "stream too long");
    try {
        std::vector<float> prob(nf);
        v->eng->probs(pcm, (int)nf, prob.data());
        std::vector<float> kept;
        std::vector<uint8_t> kinds(nf + (rem ? 1 : 0));
        for (size_t f = 0; f < nf; ++f)
            kinds[f] = (uint8_t)v->smooth->push(pcm + f * spt::kVadFrame, spt::kVadFrame, prob[f] > v->threshold, &kept);
        if (rem) {  // not a 30 ms frame: SileroVad errs, the recorder keeps it (recorder.rs:298)
            v->smooth->push_unchecked(pcm + nf * spt::kVadFrame, (int)rem, &kept);
            kinds[nf] = 1;
        }
        spt_vad_result* r = (spt_vad_result*)calloc(1, sizeof(spt_vad_result));
        if (!r) return fail(v, SPT_ERR_OOM, "host allocation failed");
        r->n_frames = (int32_t)kinds.size();
        r->n_samples = kept.size();
        r->samples = (float*)malloc(std::max<size_t>(1, kept.size()) * sizeof(float));
        r->prob = (float*)malloc(std::max<size_t>(1, nf) * sizeof(float));
        r->kind = (uint8_t*)malloc(std::max<size_t>(1, kinds.size()));
        if (!r->samples || !r->prob || !r->kind) {
            spt_vad_result_free(r);
            return fail(v, SPT_ERR_OOM, "host allocation failed");
        }
        if (!kept.empty()) memcpy(r->samples, kept.data(), kept.size() * sizeof(float));
        if (nf) memcpy(r->prob, prob.data(), nf * sizeof(float));
        if (!kinds.empty()) memcpy(r->kind, kinds.data(), kinds.size());
        r->device_ms = v->eng->last_ms();
        *out = r;
        return SPT_OK;
    } catch (const std::exception& e) {
        return fail(v, classify(e), e.what());
    }
}

void spt_vad_result_free(spt_vad_result* r) {
    if (!r) return;
    free(r->samples);
    free(r->prob);
    free(r->kind);
    free(r);
}

spt_status spt_vad_reset(spt_vad* v, int32_t reset_model_state) {
    if (!v) return SPT_ERR_INVALID_ARG;
    v->smooth->reset();
    if (reset_model_state) {
        try {
            v->eng->reset_state();
        } catch (const std::exception& e) {
            return fail(v, classify(e), e.what());
        }
    }
    return SPT_OK;
}

const char* spt_vad_last_error(const spt_vad* v) { return v ? v->err.c_str() : "null context"; }

void spt_vad_destroy(spt_vad* v) { delete v; }

}  // extern "C"
