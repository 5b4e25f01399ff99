// wait.hpp -- bounded host waits on work the engine's stream publishes.
//
// Every wait of the engine for its stream goes through wait_until(): it polls a completion
// predicate (a sequence number in mapped memory, or a HIP event), and every ~20 ms of
// waiting it also asks the stream whether it failed or drained and the RCCL communicator
// whether a peer rank reported an asynchronous error.  A wait that outlasts its timeout ends
// too.  So a dead peer rank (whose all-reduce never completes) or a faulted stream ends
// the call with a status instead of hanging every rank.  Pure host logic, templated on the
// probes so tests/test_host_logic.py drives it with scripted probes (qvq_host_wait_probe).
#pragma once
#include <chrono>
#include <string>

#include "qvq.h"

namespace qvq {

// One step of a host spin-wait: the x86 pause hint, so a polling thread leaves its core's
// other hardware thread (often the one building the level's kd-tree) its issue slots.
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

enum class StreamState { Running, Drained, Failed };
enum class CommState { None, Healthy, Failed };

// done(): the awaited work has published.  stream(msg): the stream's state (Failed fills
// msg).  comm(msg): the communicator's state (Failed fills msg).  Returns QVQ_OK, or
//   QVQ_ECOMM    the communicator reported an error, or the wait timed out with a
//                communicator present (the likely cause: a peer rank died mid-collective),
//   QVQ_EDEVICE  the stream failed, drained without publishing, or timed out alone.
template <class Done, class Stream, class Comm>
qvq_status wait_until(Done done, Stream stream, Comm comm, double timeout_s, std::string &err) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    const auto deadline = t0 + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(timeout_s));
    // hipStreamQuery submits a marker (a few us of GPU idle): consult the stream and the
    // communicator only every ~20 ms of waiting
    auto next_check = t0 + std::chrono::milliseconds(20);
    while (!done()) {
        cpu_relax();
        const auto now = clock::now();
        if (now < next_check) continue;
        std::string msg;
        const CommState cs = comm(msg);
        if (cs == CommState::Failed) {
            err = "communicator error: " + msg;
            return QVQ_ECOMM;
        }
        const StreamState ss = stream(msg);
        if (ss == StreamState::Failed) {
            err = "stream: " + msg;
            return QVQ_EDEVICE;
        }
        if (ss == StreamState::Drained) {
            if (done()) break;
            err = "the stream finished without publishing its completion";
            return QVQ_EDEVICE;
        }
        if (now >= deadline) {
            const double s = std::chrono::duration<double>(now - t0).count();
            if (cs == CommState::Healthy) {
                err = "timed out after " + std::to_string(s) + " s waiting for the stream (a peer rank stalled?)";
                return QVQ_ECOMM;
            }
            err = "timed out after " + std::to_string(s) + " s waiting for the stream";
            return QVQ_EDEVICE;
        }
        next_check = now + std::chrono::milliseconds(20);
    }
    return QVQ_OK;
}

}  // namespace qvq
