// Cost of starting and joining host threads (diagnostics for the accelerator build's
// parallel_chunks on the GPU box's CPU share). Build (from tools/native):
//   g++ -O2 -std=c++17 -pthread -o build/thread_cost thread_cost.cpp
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

int main() {
    for (int T : {2, 4, 8, 16}) {
        double best = 1e30, sum = 0;
        const int reps = 20;
        for (int r = 0; r < reps; ++r) {
            std::atomic<int> n{0};
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int c = 1; c < T; ++c) th.emplace_back([&] { n.fetch_add(1); });
            for (auto& t : th) t.join();
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            best = std::min(best, us);
            sum += us;
        }
        std::printf("threads %2d: start+join %8.1f us best, %8.1f us mean\n", T, best, sum / reps);
    }
    // effective parallelism: the same fixed work on every thread (ideal: flat time)
    for (int T : {1, 2, 4, 8, 16}) {
        std::vector<double> out(T);
        const auto t0 = std::chrono::steady_clock::now();
        auto work = [&](int c) {
            double x = 1.0 + c;
            for (int i = 0; i < 20000000; ++i) x = x * 1.0000001 + 1e-9;
            out[c] = x;
        };
        std::vector<std::thread> th;
        for (int c = 1; c < T; ++c) th.emplace_back(work, c);
        work(0);
        for (auto& t : th) t.join();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::printf("threads %2d: fixed work per thread %8.2f ms (%g)\n", T, ms, out[0]);
    }
    std::printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
}
