// host_loop.cpp — the reference's GPU render loop (src/main.cpp:290-462) as a C++
// host over the C ABI (librthost.so; include/rt_host.h).
//
// Per frame the reference uploads the camera and the light (SSBO 2 and 1,
// :328-334), dispatches the compute shader (:352-354) and, before the next frame,
// waits for it (glfwSwapBuffers; FPS = 1 / deltaTime, :290-300). This file is that
// loop with the rt_* calls that replace the GL ones, so a waited
// frame can be timed the way a C++ host would see it, without an interpreter
// between the calls. It links librtamd.so through its headers only.
#include <chrono>
#include <cstddef>

#include "../../include/rt_api.h"
#include "../../include/rt_host.h"

extern "C" int rth_render_loop_anim(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light,
                                    int width, int height, float* dst, size_t pitch, int frames, int wait_each,
                                    const FlatShape* anim, int anim_count, int anim_frames, double* frame_ms) {
    if (!ctx || !cams || ncams < 1 || !light || !dst || frames < 0 || !frame_ms) return RT_ERR_INVALID;
    if (anim && (anim_count < 1 || anim_frames < 1)) return RT_ERR_INVALID;
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    for (int i = 0; i < frames; ++i) {
        if (wait_each) t0 = clk::now();
        int rc = rt_set_camera(ctx, &cams[i % ncams]);                                        // SSBO 2
        if (rc == RT_OK) rc = rt_set_light(ctx, light);                                        // SSBO 1
        if (rc == RT_OK && anim)  // updateScene + updateBVH + their uploads (:336-346), on the device
            rc = rt_animate(ctx, anim + static_cast<size_t>(i % anim_frames) * anim_count);
        if (rc == RT_OK) rc = rt_dispatch_rows(ctx, width, height, 0, 1, 1, height, dst, pitch);  // dispatch
        if (rc == RT_OK && wait_each) rc = rt_sync(ctx);                                       // the frame's end
        if (rc != RT_OK) return rc;
        if (wait_each) frame_ms[i] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    }
    if (!wait_each) {
        const int rc = rt_sync(ctx);
        if (rc != RT_OK) return rc;
        frame_ms[0] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    }
    return RT_OK;
}

extern "C" int rth_render_loop(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light, int width,
                               int height, float* dst, size_t pitch, int frames, int wait_each, double* frame_ms) {
    return rth_render_loop_anim(ctx, cams, ncams, light, width, height, dst, pitch, frames, wait_each, nullptr, 0, 0,
                                frame_ms);
}
