// host_loop.cpp — the reference's GPU render loop (src/main.cpp:290-462) as a C++
// host over the C ABI (librthost.so; include/rt_host.h).
//
// Per frame the reference uploads the camera and the light (SSBO 2 and 1,
// :328-334), dispatches the compute shader (:352-354) and, before the next frame,
// waits for it (glfwSwapBuffers; FPS = 1 / deltaTime, :290-300). This file is that
// loop with the rt_* calls that replace the GL ones, so a waited
// frame can be timed the way a C++ host would see it, without an interpreter
// between the calls. It links librtamd.so and librtscene.so through their headers only.
#include <chrono>
#include <cstddef>

#include "../../include/rt_api.h"
#include "../../include/rt_group.h"
#include "../../include/rt_host.h"
#include "../../include/rt_scene.h"

namespace {

// The reference's own upload of an animated frame, call for call (:336-346):
// updateScene's glBufferSubData of each animated record (:981-992), updateBVH on
// the host's node objects (:1068-1077), then serializeBVH and one glBufferSubData
// of every node record (:340-345). T: a context (rt_update_*) or a group
// (rt_group_update_*, every member and frame slot).
template <class T, class Shapes, class Nodes>
int upload_animated(T* dst, Shapes update_shapes, Nodes update_nodes, FlatShape* shapes, int num_shapes,
                    const int* ids, const FlatShape* recs, int count, FlatNode* nodes, int num_nodes,
                    const int* indices, int num_indices) {
    if (!dst || !shapes || num_shapes < 0 || count < 0 || (count > 0 && (!ids || !recs)) || !nodes || num_nodes < 0)
        return RT_ERR_INVALID;
    for (int j = 0; j < count; ++j) {
        if (ids[j] < 0 || ids[j] >= num_shapes) return RT_ERR_INVALID;
        shapes[ids[j]] = recs[j];                                       // flatScene.shapes[i] = serializeShape(...)
        const int rc = update_shapes(dst, ids[j], 1, &shapes[ids[j]]);  // glBufferSubData of that one record
        if (rc != RT_OK) return rc;
    }
    if (rts_update_bvh(shapes, num_shapes, nodes, num_nodes, indices, num_indices, ids, count) != 0)  // updateBVH
        return RT_ERR_INVALID;
    return update_nodes(dst, nodes, num_nodes);  // serializeBVH + glBufferSubData of the nodes
}

}  // namespace

extern "C" int rth_upload_animated(rt_ctx* ctx, FlatShape* shapes, int num_shapes, const int* ids,
                                   const FlatShape* recs, int count, FlatNode* nodes, int num_nodes, const int* indices,
                                   int num_indices) {
    return upload_animated(ctx, rt_update_shapes, rt_update_nodes, shapes, num_shapes, ids, recs, count, nodes,
                           num_nodes, indices, num_indices);
}

// The same over a multi-GPU group (include/rt_group.h): every local member and frame
// slot is given each call.
extern "C" int rth_group_upload_animated(rt_group* g, FlatShape* shapes, int num_shapes, const int* ids,
                                         const FlatShape* recs, int count, FlatNode* nodes, int num_nodes,
                                         const int* indices, int num_indices) {
    return upload_animated(g, rt_group_update_shapes, rt_group_update_nodes, shapes, num_shapes, ids, recs, count,
                           nodes, num_nodes, indices, num_indices);
}

namespace {

struct RefUpload {  // rth_render_loop_ref's scene, moved by the reference's upload
    FlatShape* shapes;
    int num_shapes;
    const int* ids;
    int count;
    const FlatShape* anim;
    int anim_frames;
    FlatNode* nodes;
    int num_nodes;
    const int* indices;
    int num_indices;
};

struct Rows {  // the rows one dispatch renders (rt_dispatch_rows_ex)
    int y0, stripe, period, out_rows, format;
};

int render_loop(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light, int width, int height,
                float* dst, size_t pitch, int frames, int wait_each, const FlatShape* anim, int anim_count,
                int anim_frames, const RefUpload* ref, double* frame_ms, const Rows* rows = nullptr) {
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
        if (rc == RT_OK && ref)  // the same, as the reference uploads it
            rc = rth_upload_animated(ctx, ref->shapes, ref->num_shapes, ref->ids,
                                     ref->anim + static_cast<size_t>(i % ref->anim_frames) * ref->count, ref->count,
                                     ref->nodes, ref->num_nodes, ref->indices, ref->num_indices);
        if (rc == RT_OK)  // dispatch
            rc = rows ? rt_dispatch_rows_ex(ctx, width, height, rows->y0, rows->stripe, rows->period, rows->out_rows,
                                            dst, pitch, rows->format)
                      : rt_dispatch_rows(ctx, width, height, 0, 1, 1, height, dst, pitch);
        if (rc == RT_OK && wait_each) rc = rt_sync_frame(ctx);                                 // the frame's end
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

}  // namespace

extern "C" int rth_render_loop_anim(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light,
                                    int width, int height, float* dst, size_t pitch, int frames, int wait_each,
                                    const FlatShape* anim, int anim_count, int anim_frames, double* frame_ms) {
    return render_loop(ctx, cams, ncams, light, width, height, dst, pitch, frames, wait_each, anim, anim_count,
                       anim_frames, nullptr, frame_ms);
}

extern "C" int rth_render_loop(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light, int width,
                               int height, float* dst, size_t pitch, int frames, int wait_each, double* frame_ms) {
    return render_loop(ctx, cams, ncams, light, width, height, dst, pitch, frames, wait_each, nullptr, 0, 0, nullptr,
                       frame_ms);
}

extern "C" int rth_render_loop_ref(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light, int width,
                                   int height, float* dst, size_t pitch, int frames, int wait_each, FlatShape* shapes,
                                   int num_shapes, const int* ids, int count, const FlatShape* anim, int anim_frames,
                                   FlatNode* nodes, int num_nodes, const int* indices, int num_indices,
                                   double* frame_ms) {
    if (!shapes || !ids || !anim || count < 1 || anim_frames < 1 || !nodes) return RT_ERR_INVALID;
    const RefUpload ref{shapes, num_shapes, ids, count, anim, anim_frames, nodes, num_nodes, indices, num_indices};
    return render_loop(ctx, cams, ncams, light, width, height, dst, pitch, frames, wait_each, nullptr, 0, 0, &ref,
                       frame_ms);
}

extern "C" int rth_render_rows_loop(rt_ctx* ctx, const FlatCamera* cams, int ncams, const FlatLight* light, int width,
                                    int height, int y0, int stripe, int period, int out_rows, int format, float* dst,
                                    size_t pitch, int frames, int wait_each, double* frame_ms) {
    const Rows rows{y0, stripe, period, out_rows, format};
    return render_loop(ctx, cams, ncams, light, width, height, dst, pitch, frames, wait_each, nullptr, 0, 0, nullptr,
                       frame_ms, &rows);
}
