// wait_check: the bounded wait behind rt_group_sync (csrc/group_wait.h), driven
// with fake stream/communicator queries on the CPU. Prints one line per case and
// exits non-zero on the first mismatch.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "../../opengl-ray-tracer_amd/csrc/group_wait.h"

using namespace rtg;

static int fails = 0;
#define EXPECT(c)                                               \
    do {                                                        \
        if (!(c)) {                                             \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                            \
        }                                                       \
    } while (0)

int main() {
    using clk = std::chrono::steady_clock;
    // finishes after 5 polls
    int n = 0;
    EXPECT(wait_bounded([&] { return ++n < 5 ? 1 : 0; }, [] { return false; }, 1000.0) == kWaitDone);
    EXPECT(n == 5);
    // a fan-in that never completes: the deadline, not a hang
    auto t0 = clk::now();
    EXPECT(wait_bounded([] { return 1; }, [] { return false; }, 50.0) == kWaitTimeout);
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    EXPECT(ms >= 50.0 && ms < 2000.0);
    // the communicator reports an asynchronous error while work is outstanding
    int k = 0;
    EXPECT(wait_bounded([] { return 1; }, [&] { return ++k >= 3; }, 0.0) == kWaitCommError);
    // a device error from a stream query
    EXPECT(wait_bounded([] { return -1; }, [] { return false; }, 1000.0) == kWaitDeviceError);
    // finished work wins over a late error report
    EXPECT(wait_bounded([] { return 0; }, [] { return true; }, 1000.0) == kWaitDone);
    // a frame that ends 300 us in is seen within a poll, not after a nap (round 3's
    // back-off slept 20 -> 320 us between polls: a 0.27 ms frame was seen at ~0.35 ms)
    // (median of 21 waits: a loaded host may deschedule the polling thread now and then)
    std::vector<double> late;
    for (int rep = 0; rep < 21; ++rep) {
        const auto t1 = clk::now();
        const auto end = t1 + std::chrono::microseconds(300);
        EXPECT(wait_bounded([&] { return clk::now() < end ? 1 : 0; }, [] { return false; }, 1000.0) == kWaitDone);
        late.push_back(std::chrono::duration<double, std::micro>(clk::now() - end).count());
    }
    std::sort(late.begin(), late.end());
    const double late_max = late[late.size() / 2];
    EXPECT(late_max < 50.0);
    // past the spin phase the wait naps (a hung fan-in does not burn a core): a 50 ms
    // timeout with a 5 ms spin polls far fewer times than a busy loop would
    long polls = 0;
    EXPECT(wait_bounded([&] { ++polls; return 1; }, [] { return false; }, 50.0, 5.0) == kWaitTimeout);
    std::printf("%s (%.1f ms timeout case, frame end seen a median %.1f us late, %ld polls in 50 ms)\n",
                fails ? "wait_check FAILED" : "wait_check ok", ms, late_max, polls);
    return fails ? 1 : 0;
}
