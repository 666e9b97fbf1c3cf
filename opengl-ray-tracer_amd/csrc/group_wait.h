// group_wait.h — the bounded wait behind rt_group_sync (csrc/rt_group.hip).
//
// A multi-GPU frame ends in an RCCL fan-in: if a peer dies or never posts its
// send, the receiving kernel spins for ever and a plain hipStreamSynchronize
// never returns. rt_group_sync therefore polls instead: every stream of the
// group with hipStreamQuery, the communicator with ncclCommGetAsyncError, and a
// deadline. Host-only and free of HIP/RCCL types so that a CPU test
// (tests/native/wait_check.cpp) can drive it with fake queries.
#ifndef RT_GROUP_WAIT_H
#define RT_GROUP_WAIT_H

#include <chrono>
#include <thread>

namespace rtg {

enum WaitResult { kWaitDone = 0, kWaitTimeout = 1, kWaitCommError = 2, kWaitDeviceError = 3 };

// pending(): >0 while work is outstanding, 0 when everything finished, <0 on a
// device error. comm_error(): true once the communicator reports an
// asynchronous error. Polls with a back-off from 20 us to 1 ms; gives up after
// timeout_ms (<= 0: no deadline).
template <class Pending, class CommError>
WaitResult wait_bounded(Pending pending, CommError comm_error, double timeout_ms) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto nap = std::chrono::microseconds(20);
    for (;;) {
        const int p = pending();
        if (p < 0) return kWaitDeviceError;
        if (p == 0) return kWaitDone;
        if (comm_error()) return kWaitCommError;
        if (timeout_ms > 0 &&
            std::chrono::duration<double, std::milli>(clk::now() - t0).count() > timeout_ms)
            return kWaitTimeout;
        std::this_thread::sleep_for(nap);
        if (nap < std::chrono::microseconds(1000)) nap *= 2;
    }
}

}  // namespace rtg

#endif
