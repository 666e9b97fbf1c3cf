// wait_probe: how the host best sees a kernel end (the waited frame's turn-around).
// For an empty kernel and for a 235-us kernel (a wall-clock wait, the car frame's
// length), the launch-to-seen time of:
//   sync   hipStreamSynchronize
//   squery polling hipStreamQuery
//   equery hipEventRecord after the kernel, polling hipEventQuery
//   esync  hipEventRecord + hipEventSynchronize
// Run with and without ROC_ACTIVE_WAIT_TIMEOUT to see the runtime's wait policy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_wait(unsigned long long ticks) {
    if (ticks == 0) return;
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
}

using clk = std::chrono::steady_clock;
static double dus(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e;
    hipEventCreateWithFlags(&e, hipEventDisableTiming);
    const char* env = std::getenv("ROC_ACTIVE_WAIT_TIMEOUT");
    for (unsigned long long ticks : {0ull, 23500ull}) {  // wall clock 100 MHz: 0 and 235 us
        for (int mode = 0; mode < 4; ++mode) {
            std::vector<double> t;
            for (int i = 0; i < 300; ++i) {
                const auto a = clk::now();
                hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, ticks);
                if (mode == 0) {
                    hipStreamSynchronize(s);
                } else if (mode == 1) {
                    while (hipStreamQuery(s) == hipErrorNotReady) {
                    }
                } else if (mode == 2) {
                    hipEventRecord(e, s);
                    while (hipEventQuery(e) == hipErrorNotReady) {
                    }
                } else {
                    hipEventRecord(e, s);
                    hipEventSynchronize(e);
                }
                if (i >= 50) t.push_back(dus(a, clk::now()));
            }
            static const char* names[4] = {"sync", "squery", "equery", "esync"};
            std::printf("ROC_ACTIVE_WAIT_TIMEOUT=%s kernel %4.0f us  %-6s %.1f us\n", env ? env : "(unset)", ticks / 100.0,
                        names[mode], med(t));
        }
    }
    return 0;
}
