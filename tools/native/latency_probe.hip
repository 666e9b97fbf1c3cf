// latency_probe: the fixed cost of one waited frame outside the render kernel.
//   1. hipStreamQuery on an idle stream (host cost per poll)
//   2. an empty kernel: launch + poll until done (the runtime's round trip)
//   3. the same with hipStreamSynchronize
//   4. a 8x8-pixel car frame through the C ABI: rt_set_camera + rt_set_light +
//      rt_dispatch_rows + rt_sync (the renderer's fixed cost per frame)
//   5. rt_dispatch_rows's host time alone (GPU busy with the previous frames)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/native/build/latency_probe tools/native/latency_probe.hip
//        -Lopengl-ray-tracer_amd/lib -lrtamd -lrtscene -Wl,-rpath,...
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_scene.h"

__global__ void k_empty() {}

using clk = std::chrono::steady_clock;
static double dus(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<double> q, poll_v, sync_v, frame, host;
    for (int i = 0; i < 2000; ++i) {
        auto a = clk::now();
        (void)hipStreamQuery(s);
        q.push_back(dus(a, clk::now()));
    }
    for (int i = 0; i < 500; ++i) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        while (hipStreamQuery(s) == hipErrorNotReady) {
        }
        poll_v.push_back(dus(a, clk::now()));
    }
    for (int i = 0; i < 500; ++i) {
        auto a = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
        hipStreamSynchronize(s);
        sync_v.push_back(dus(a, clk::now()));
    }
    // the car through the C ABI
    struct rts_scene* sc = rts_new();
    rts_generate(sc, 3, 0, 16.f / 9.f);
    int S = 0, N = 0, I = 0;
    rts_counts(sc, &S, &N, &I);
    std::vector<FlatShape> shapes(S);
    std::vector<FlatNode> nodes(N);
    std::vector<int> idx(I);
    FlatCamera cam;
    FlatLight light;
    rts_serialize(sc, shapes.data(), nodes.data(), idx.data(), &cam, &light);
    rt_ctx* c = nullptr;
    if (rt_create(&c, 0) != RT_OK) return 1;
    rt_upload_scene(c, shapes.data(), S, nodes.data(), N, idx.data(), I);
    rt_params p{1920.f, 1080.f, 3, 1, 0, 0};
    rt_set_params(c, &p);
    rt_set_kernel_timing(c, 0);
    rt_set_latency_mode(c, 1);
    float* dst = nullptr;
    hipMalloc(&dst, 1920 * 1080 * 16);
    for (int i = 0; i < 600; ++i) {
        auto a = clk::now();
        rt_set_camera(c, &cam);
        rt_set_light(c, &light);
        rt_dispatch_rows(c, 8, 8, 0, 1, 1, 8, dst, 8 * 16);  // one 8x8 tile
        rt_sync(c);
        if (i >= 100) frame.push_back(dus(a, clk::now()));
    }
    for (int i = 0; i < 300; ++i) {  // host time of a 1080p dispatch while the GPU is busy
        rt_set_camera(c, &cam);
        rt_set_light(c, &light);
        auto a = clk::now();
        rt_dispatch_rows(c, 1920, 1080, 0, 1, 1, 1080, dst, 1920 * 16);
        host.push_back(dus(a, clk::now()));
    }
    rt_sync(c);
    std::printf("hipStreamQuery idle: %.2f us; empty kernel + poll: %.1f us; + hipStreamSynchronize: %.1f us; "
                "8x8 car frame via the C ABI + rt_sync: %.1f us; rt_dispatch_rows host time (1080p): %.1f us\n",
                med(q), med(poll_v), med(sync_v), med(frame), med(host));
    rt_destroy(c);
    rts_free(sc);
    return 0;
}
