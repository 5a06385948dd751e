// multi.cpp -- multi-GPU replica parallelism behind the C ABI.
//
// Whisper windows are independent, so N GPUs run N independent engines with no data-path
// collective.  The one collective is at load: the weight arena of device 0 is broadcast over
// RCCL (xGMI) into the arenas of the others, whose layout is the same pure function of
// (model, dtype).  Two ways in:
//
//  * one process driving N devices (a Rust host: the app's TranscriptionManager owns one
//    engine, transcription.rs:29-47): spt_ctx_create_replicas loads device 0 and runs one
//    grouped ncclBroadcast over a ncclCommInitAll communicator straight into every arena;
//    spt_transcribe_batch_replicas shards a batch over the contexts, one host thread each.
//  * one process per GPU (torchrun, bench.py): spt_weights_arena exposes the arena so the
//    rank's collective (torch.distributed over RCCL) writes rank 0's bytes straight into it,
//    then spt_weights_commit marks the context usable.
//
// RCCL is opened at run time (dlopen) so that the library has no link-time dependency on it and
// a process that never asks for replicas never loads it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "capi_internal.h"
#include "common.h"

namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclBroadcast) bcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    bool ok() const { return init_all && bcast && group_start && group_end && destroy && err; }
};

const Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            x.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (x.h) break;
        }
        if (!x.h) return x;
        x.init_all = (decltype(x.init_all))dlsym(x.h, "ncclCommInitAll");
        x.bcast = (decltype(x.bcast))dlsym(x.h, "ncclBroadcast");
        x.group_start = (decltype(x.group_start))dlsym(x.h, "ncclGroupStart");
        x.group_end = (decltype(x.group_end))dlsym(x.h, "ncclGroupEnd");
        x.destroy = (decltype(x.destroy))dlsym(x.h, "ncclCommDestroy");
        x.err = (decltype(x.err))dlsym(x.h, "ncclGetErrorString");
        return x;
    }();
    return r;
}

void set_err(char* buf, size_t len, const std::string& msg) {
    if (buf && len) {
        strncpy(buf, msg.c_str(), len - 1);
        buf[len - 1] = 0;
    }
}

// contiguous balanced shard [begin, end) of n items for rank r of w (spittle_amd.dist.shard_range)
void shard(size_t n, size_t w, size_t r, size_t* b, size_t* e) {
    const size_t base = n / w, rem = n % w;
    *b = r * base + std::min(r, rem);
    *e = *b + base + (r < rem ? 1 : 0);
}

}  // namespace

extern "C" {

spt_status spt_weights_arena(spt_ctx* ctx, void** dev_ptr, size_t* bytes) {
    if (!ctx || !dev_ptr || !bytes) return spt_fail(ctx, SPT_ERR_INVALID_ARG, "null argument");
    *dev_ptr = ctx->eng->weight_arena();
    *bytes = (size_t)ctx->eng->weight_bytes();
    return SPT_OK;
}

spt_status spt_weights_commit(spt_ctx* ctx) {
    if (!ctx) return SPT_ERR_INVALID_ARG;
    try {
        ctx->eng->commit_weights();
        return SPT_OK;
    } catch (const std::exception& e) {
        return spt_fail(ctx, spt_classify(e), e.what());
    }
}

spt_status spt_ctx_create_replicas(const char* model_spec, const spt_model_params* params, const int32_t* devices,
                                   int32_t n_devices, spt_ctx** out, double* bcast_ms, char* err, size_t errlen) {
    if (!model_spec || !devices || !out || n_devices < 1 || n_devices > 64) {
        set_err(err, errlen, "bad argument");
        return SPT_ERR_INVALID_ARG;
    }
    for (int i = 0; i < n_devices; ++i) {
        out[i] = nullptr;
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j]) {
                set_err(err, errlen, "a device appears twice in the replica list");
                return SPT_ERR_INVALID_ARG;
            }
    }
    if (bcast_ms) *bcast_ms = 0.0;
    spt_model_params mp;
    spt_default_model_params(&mp);
    if (params) mp = *params;
    auto cleanup = [&] {
        for (int i = 0; i < n_devices; ++i) {
            spt_ctx_destroy(out[i]);
            out[i] = nullptr;
        }
    };
    // device 0 loads (file parse + device dequantisation, or synthetic generation); the others
    // allocate their arenas only
    for (int i = 0; i < n_devices; ++i) {
        spt_model_params p = mp;
        p.device = devices[i];
        p.flags = i == 0 ? (mp.flags & ~SPT_MODEL_WEIGHTS_EXTERNAL) : (mp.flags | SPT_MODEL_WEIGHTS_EXTERNAL);
        const spt_status s = spt_ctx_create(model_spec, &p, &out[i], err, errlen);
        if (s != SPT_OK) {
            cleanup();
            return s;
        }
    }
    if (n_devices == 1) return SPT_OK;
    const Rccl& r = rccl();
    if (!r.ok()) {
        cleanup();
        set_err(err, errlen, "RCCL (librccl.so.1) could not be loaded");
        return SPT_ERR_DEVICE;
    }
    std::vector<ncclComm_t> comms(n_devices, nullptr);
    std::vector<int> devs(devices, devices + n_devices);
    ncclResult_t nr = r.init_all(comms.data(), n_devices, devs.data());
    if (nr != ncclSuccess) {
        cleanup();
        set_err(err, errlen, std::string("ncclCommInitAll: ") + r.err(nr));
        return SPT_ERR_DEVICE;
    }
    std::vector<hipStream_t> st(n_devices, nullptr);
    std::string msg;
    const size_t bytes = (size_t)out[0]->eng->weight_bytes();
    for (int i = 0; i < n_devices && msg.empty(); ++i) {
        if ((size_t)out[i]->eng->weight_bytes() != bytes) msg = "replicas disagree on the weight arena size";
        else if (hipSetDevice(devices[i]) != hipSuccess || hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) != hipSuccess)
            msg = "stream creation failed";
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (msg.empty()) {
        r.group_start();
        for (int i = 0; i < n_devices; ++i) {
            void* a = out[i]->eng->weight_arena();
            (void)hipSetDevice(devices[i]);
            nr = r.bcast(a, a, bytes, ncclUint8, 0, comms[i], st[i]);
            if (nr != ncclSuccess && msg.empty()) msg = std::string("ncclBroadcast: ") + r.err(nr);
        }
        nr = r.group_end();
        if (nr != ncclSuccess && msg.empty()) msg = std::string("ncclGroupEnd: ") + r.err(nr);
        for (int i = 0; i < n_devices; ++i)
            if (st[i] && hipStreamSynchronize(st[i]) != hipSuccess && msg.empty()) msg = "broadcast stream failed";
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int i = 0; i < n_devices; ++i) {
        if (st[i]) {
            (void)hipSetDevice(devices[i]);
            (void)hipStreamDestroy(st[i]);
        }
        if (comms[i]) r.destroy(comms[i]);
    }
    if (msg.empty())
        for (int i = 1; i < n_devices; ++i)
            if (spt_weights_commit(out[i]) != SPT_OK) msg = "weight commit failed";
    if (!msg.empty()) {
        cleanup();
        set_err(err, errlen, msg);
        return SPT_ERR_DEVICE;
    }
    if (bcast_ms) *bcast_ms = ms;
    return SPT_OK;
}

spt_status spt_transcribe_batch_replicas(spt_ctx* const* ctxs, int32_t n_ctx, const float* const* pcm,
                                         const size_t* n_samples, size_t batch, const spt_infer_params* params,
                                         spt_result** out) {
    if (!ctxs || n_ctx < 1 || !out || (batch && (!pcm || !n_samples))) return SPT_ERR_INVALID_ARG;
    for (int i = 0; i < n_ctx; ++i)
        if (!ctxs[i]) return SPT_ERR_INVALID_ARG;
    for (size_t u = 0; u < batch; ++u) out[u] = nullptr;
    std::vector<spt_status> st(n_ctx, SPT_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n_ctx; ++i) {
        size_t b, e;
        shard(batch, (size_t)n_ctx, (size_t)i, &b, &e);
        if (e <= b) continue;
        // every context selects its own device on entry; the threads share nothing
        th.emplace_back([&, i, b, e] { st[i] = spt_transcribe_batch(ctxs[i], pcm + b, n_samples + b, e - b, params, out + b); });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < n_ctx; ++i)
        if (st[i] != SPT_OK) {
            for (size_t u = 0; u < batch; ++u) {
                spt_result_free(out[u]);
                out[u] = nullptr;
            }
            if (i != 0) ctxs[0]->err = "replica " + std::to_string(i) + ": " + ctxs[i]->err;
            return st[i];
        }
    return SPT_OK;
}

}  // extern "C"
