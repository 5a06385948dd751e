// capi_internal.h -- the context behind the opaque spt_ctx handle, shared by the C-ABI files.
#pragma once
#include <exception>
#include <memory>
#include <string>

#include "../../include/spittle_hip.h"
#include "engine.h"
#include "vocab.h"

struct spt_ctx {
    std::unique_ptr<spt::Engine> eng;
    std::unique_ptr<spt::Vocab> vocab;  // ggml models; synthetic models have none
    std::string spec;
    std::string err;
};

// record msg as the context's last error and return s
spt_status spt_fail(spt_ctx* c, spt_status s, const std::string& msg);
// status code of an exception thrown below the boundary
spt_status spt_classify(const std::exception& e);
