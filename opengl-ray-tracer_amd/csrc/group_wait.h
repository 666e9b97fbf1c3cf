// group_wait.h — the bounded waits behind rt_sync (csrc/rt_kernels.hip) and
// rt_group_sync (csrc/rt_group.hip).
//
// A multi-GPU frame ends in an RCCL fan-in: if a peer dies or never posts its
// send, the receiving kernel spins for ever and a plain hipStreamSynchronize
// never returns. rt_group_sync therefore polls instead: every stream of the
// group with hipStreamQuery, the communicator with ncclCommGetAsyncError, and a
// deadline. Host-only and free of HIP/RCCL types so that a CPU test
// (tests/native/wait_check.cpp) can drive it with fake queries.
//
// Polling cadence. A frame is a fraction of a millisecond (the 1080p car:
// ~0.25 ms on one GPU, ~0.04 ms per rank's share at 8 GPUs), so the first
// kSpinMs of a wait poll back to back, yielding the core between polls:
// the frame's end is seen within a poll (~1-2 us) instead of after a nap.
// Round 3's back-off slept 20 -> 40 -> ... -> 320 us between polls, which
// put ~0.1-0.3 ms on every waited frame (1-rank strong frame 0.351 ms
// against 0.268 ms direct, profiles/r03w_bench_strong_1rank.json). Past
// kSpinMs the wait is long anyway (a big frame, or a stalled peer), and it
// naps with the old back-off so that a hung fan-in does not burn a core for
// the whole timeout.
#ifndef RT_GROUP_WAIT_H
#define RT_GROUP_WAIT_H

#include <chrono>
#include <thread>

namespace rtg {

enum WaitResult { kWaitDone = 0, kWaitTimeout = 1, kWaitCommError = 2, kWaitDeviceError = 3 };

constexpr double kSpinMs = 20.0;  // back-to-back polls for this long, then naps

// pending(): >0 while work is outstanding, 0 when everything finished, <0 on a
// device error. comm_error(): true once the communicator reports an
// asynchronous error. Spins (yielding) for spin_ms, then polls with a back-off
// from 20 us to 1 ms; gives up after timeout_ms (<= 0: no deadline).
template <class Pending, class CommError>
WaitResult wait_bounded(Pending pending, CommError comm_error, double timeout_ms, double spin_ms = kSpinMs) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto nap = std::chrono::microseconds(20);
    for (unsigned polls = 0;; ++polls) {
        const int p = pending();
        if (p < 0) return kWaitDeviceError;
        if (p == 0) return kWaitDone;
        // the communicator's error state is a host-side read: every 16th poll while spinning
        const bool spinning_phase = (polls & 15u) != 0;
        const double el = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        const bool spinning = el < spin_ms;
        if ((!spinning || !spinning_phase) && comm_error()) return kWaitCommError;
        if (timeout_ms > 0 && el > timeout_ms) return kWaitTimeout;
        if (spinning) {
            std::this_thread::yield();
            continue;
        }
        std::this_thread::sleep_for(nap);
        if (nap < std::chrono::microseconds(1000)) nap *= 2;
    }
}

}  // namespace rtg

#endif
