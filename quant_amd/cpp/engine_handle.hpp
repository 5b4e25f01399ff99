// One engine context per host thread for the C++ API (include/qvq.h underneath).
#pragma once
#include <stdexcept>
#include <string>

#include "qvq.h"

namespace quant_amd {

class EngineHandle {
public:
    static qvq_ctx *get();   // creates the context on first use (device QVQ_DEVICE, default 0)
    static void check(qvq_status st, const char *what);   // throws std::runtime_error
};

}  // namespace quant_amd
