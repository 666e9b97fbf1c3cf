/*
 * rt_api.h — C ABI of the MI355X renderer (librtamd.so).
 *
 * This is the drop-in for the reference's GPU operator boundary: the GL compute
 * program, its SSBO bindings, its uniforms and glDispatchCompute. Each entry
 * point names the reference call it replaces. Plain pointers and sizes only;
 * every function returns an int status (RT_OK = 0, negative on error) and never
 * throws across the boundary (the reference prints shader errors and carries
 * on, src/computeShader.hpp:64-79; here the caller gets a code).
 *
 * Threading: one rt_ctx per device. A context is not thread-safe; different
 * contexts may be driven from different threads. All work of a context is
 * ordered on one HIP stream (its own, or the caller's via rt_set_stream).
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>
#include "rt_flat.h"

#ifdef __cplusplus
extern "C" {
#endif

struct rt_ctx; /* opaque: one per device */

enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,   /* bad argument (null pointer, negative size, bad rows)   */
    RT_ERR_DEVICE = -2,    /* a HIP runtime call failed                              */
    RT_ERR_NO_MEMORY = -3, /* device allocation failed                               */
    RT_ERR_NO_SCENE = -4,  /* dispatch before rt_upload_scene / camera / light       */
    RT_ERR_BVH = -5,       /* node/index arrays are out of range or too deep         */
    RT_ERR_NO_DEVICE = -6, /* no HIP device with that ordinal                        */
    RT_ERR_COMM = -7,      /* an RCCL call failed (rt_group.h)                       */
    RT_ERR_TIMEOUT = -8    /* a group's frames did not finish in time (rt_group.h)   */
};

/* Uniforms of gpu_shader.comp:126-130, set by src/main.cpp:357-361.
 * Applied AT the next dispatch (the reference sets them after the dispatch, so
 * its frame k uses frame k-1's values and frame 0 uses zeros). */
typedef struct rt_params {
    float resX, resY;        /* screenRes; pixel NDC and background use these        */
    int maxBounces;          /* closest-hit bounces per pixel, >= 0                  */
    int useBVH;              /* 1: BVH traversal branch, 0: brute-force branch       */
    int useFresnel;          /* Fresnel-weighted reflections                         */
    int useMollerTrumbore;   /* triangle test: 1 Moller-Trumbore, 0 barycentric      */
} rt_params;

/* Traversal kernel variants (all produce the same image). */
enum rt_kernel {
    RT_KERNEL_AUTO = 0,      /* pick the fastest for the uploaded scene               */
    RT_KERNEL_LANE = 1,      /* one ray per lane, per-lane LDS stack (reference walk) */
    RT_KERNEL_PACKET = 2,    /* wave64 packet walk, wave-uniform stack + active mask  */
    RT_KERNEL_ACCEL = 3      /* packet walk + exact-result leaf accelerator (default  */
                             /* for BVH + barycentric; falls back to PACKET otherwise)*/
};

/* Accelerator statistics of the uploaded scene (rt_accel_info). */
typedef struct rt_accel_info {
    int built;               /* 1 if the accelerator is in use for this scene         */
    int local_nodes;         /* local BVH nodes inside large reference leaves         */
    int local_leaves;
    int bounded_prims;       /* shapes under a conservative box                       */
    int always_prims;        /* shapes tested whenever their leaf is entered          */
    int max_stack;           /* worst-case wave stack entries                          */
    int last_kernel;         /* rt_kernel of the latest render dispatch               */
    int scene_tree;          /* 1 if the scene tree is built (rt_set_tree)             */
    int scene_nodes;         /* its wide nodes                                         */
    int scene_items;         /* its leaves (shapes of one reference leaf each)         */
    int scene_height;        /* its binary height                                      */
    int tree_nested;         /* the reference tree's child boxes lie in their parents' */
    int record_bytes;        /* device records the accelerated kernel reads: nodes,   */
                             /* items, shapes, materials (its compulsory scene bytes)  */
} rt_accel_info;

/* Work counted on the reference's own traversal (gpu_shader.comp:380-430 and
 * :523-580) — what the reference shader would load. Filled by
 * rt_collect_stats; used for Mrays/s and the algorithmic-bytes roofline. */
typedef struct rt_stats {
    uint64_t pixels;              /* pixels shaded                                  */
    uint64_t closest_rays;        /* closest-hit traversals (primary + reflection)  */
    uint64_t shadow_rays;         /* shadow traversals                              */
    uint64_t node_visits;         /* FlatNode records popped and box-tested         */
    uint64_t bvh_tests[4];        /* leaf primitive tests by type (BVH branch)      */
    uint64_t brute_tests[4];      /* primitive tests by type (brute-force branch)   */
    uint64_t closest_updates;     /* closest-hit record updates (material fetches)  */
    uint64_t hits;                /* bounces that hit a shape                       */
} rt_stats;

/* ComputeShader("gpu_shader.comp") + the RGBA32F image (src/computeShader.hpp:30-83,
 * src/main.cpp:182-195). Selects HIP device `device`. */
int rt_create(struct rt_ctx** out, int device);
int rt_destroy(struct rt_ctx* ctx);

/* Order all work of the context on a caller stream (hipStream_t; NULL = own stream). */
int rt_set_stream(struct rt_ctx* ctx, void* hip_stream);

/* SSBO 3 (shapes), 4 (nodes), 5 (bvhIndices) (src/main.cpp:256-275). The root
 * is node N-1 as in gpu_shader.comp:386. Copies to HBM and re-lays the records
 * out for the kernels; the caller keeps ownership. N == 0 is allowed (the BVH
 * branch then sees no shape). Returns RT_ERR_BVH for child/index out of range. */
int rt_upload_scene(struct rt_ctx* ctx, const FlatShape* shapes, int num_shapes,
                    const FlatNode* nodes, int num_nodes, const int* indices, int num_indices);

/* Partial re-upload of shapes [first, first+count) (glBufferSubData in updateScene,
 * src/main.cpp:981-992). Node boxes are not touched (the reference's are not either,
 * until it re-uploads them). The host array may be reused when the call returns. */
int rt_update_shapes(struct rt_ctx* ctx, int first, int count, const FlatShape* shapes);

/* Re-upload of all nodes with the same topology (src/main.cpp:340-345, after
 * updateBVH + serializeBVH); RT_ERR_BVH if the topology differs.
 *
 * Both calls only write the context's host copies and return; the next operation
 * that reads the device scene (a dispatch, rt_collect_stats, rt_read_nodes,
 * rt_build_lbvh, rt_animate) applies everything written since as ONE device refit
 * on the context's stream: the moved shapes' records, the boxes of the accelerator
 * above them, and every copy of the node boxes. So the reference's loop -- one
 * rt_update_shapes per animated record, then one rt_update_nodes -- costs one small
 * kernel per frame, not one rebuild per call. The accelerator is rebuilt on the host
 * only when a moved shape's kind of bound changed (the frame is exact before that
 * too: the refit enters every box above it) or the new node boxes no longer nest
 * (the scene tree's condition, rt_set_tree). rt_debug_refits / rt_debug_anim_rebuilds
 * count the two outcomes. */
int rt_update_nodes(struct rt_ctx* ctx, const FlatNode* nodes, int num_nodes);

/* Device-side animation. Replaces the reference's
 * per-frame CPU path: updateScene + updateBVH + serializeBVH + the two
 * glBufferSubData calls (src/main.cpp:336-346, 981-992, 1068-1077).
 *
 * rt_set_animated marks the shapes the host animates: the reference's
 * animatedIndices / Shape::animated (src/main.cpp:120, 600-616, 706-708).
 * ids must be distinct and in [0, num_shapes); count 0 clears the set.
 * The set holds until the next rt_upload_scene.
 *
 * rt_animate uploads their new records: shapes[i] is shape ids[i]. On the
 * device it then grows every node whose shape set lists an animated shape to
 * include the shape, exactly as updateBVH does. That means the leaf and every
 * node above it, growToInclude (src/BoundingBox.hpp:44-95), grow-only.
 * The accelerator's conservative boxes are refit along with the node boxes, in
 * one kernel launch per call (with any rt_update_shapes / rt_update_nodes pending).
 * A moved shape whose kind of bound changes (a triangle that becomes too thin to
 * bound, a sphere whose radius becomes infinite) is entered through every box
 * above it until the host rebuilds the accelerator, which the refit requests.
 * The frame is identical either way. The host array may be reused when the call
 * returns. RT_ERR_INVALID if no set is marked.
 *
 * rt_read_nodes copies the current node records to the host, including the
 * boxes rt_animate grew. num_nodes must match the scene's node count. */
int rt_set_animated(struct rt_ctx* ctx, const int* ids, int count);
int rt_animate(struct rt_ctx* ctx, const FlatShape* shapes);
int rt_read_nodes(struct rt_ctx* ctx, FlatNode* nodes, int num_nodes);

/* SSBO 2 and 1 (src/main.cpp:328-334). */
int rt_set_camera(struct rt_ctx* ctx, const FlatCamera* camera);
int rt_set_light(struct rt_ctx* ctx, const FlatLight* light);

/* The five uniforms (src/main.cpp:357-361). */
int rt_set_params(struct rt_ctx* ctx, const rt_params* params);

/* Kernel variant; RT_KERNEL_AUTO by default. */
int rt_set_kernel(struct rt_ctx* ctx, int kernel);

/* glDispatchCompute(W,H,1) + glMemoryBarrier (src/main.cpp:352-354) into the
 * context's own W x H RGBA32F surface, rows [y0, y1). Stream-ordered, async. */
int rt_dispatch(struct rt_ctx* ctx, int width, int height, int y0, int y1);

/* Same into a caller-owned device surface (for tiling and RCCL gathers).
 * Row-stripe mapping: output row r (0-based, r < out_rows) holds image row
 *   y = y0 + (r / stripe) * stripe * step + (r % stripe)
 * so step = 1 renders the contiguous band [y0, y0+out_rows) and step = P with
 * y0 = k*stripe renders the k-th of P interleaved stripe sets. Rows with
 * y >= height are left untouched. `pitch` is in bytes (>= 16*width). */
int rt_dispatch_rows(struct rt_ctx* ctx, int width, int height, int y0, int stripe,
                     int step, int out_rows, float* dst, size_t pitch);

/* rt_dispatch_rows with an output format: RT_FORMAT_RGBA32F (16 B per pixel, as
 * the reference's image2D rgba32f) or RT_FORMAT_RGB32F (12 B per pixel, packed;
 * the alpha the reference stores is always 1, gpu_shader.comp:437,623). The
 * multi-GPU gather (rt_group.h) sends RGB32F: 25 % fewer bytes over xGMI.
 * pitch >= 12*width and 4-byte aligned for RGB32F.
 * RT_FORMAT_RGBA32F_IMAGE: RGBA32F written at each row's IMAGE row y, not at its
 * compact row r: dst is the whole width x height surface (pitch >= 16*width),
 * and rows the call does not render are left untouched. rt_group's rank 0
 * renders its stripes straight into the gathered frame this way. */
enum rt_format { RT_FORMAT_RGBA32F = 0, RT_FORMAT_RGB32F = 1, RT_FORMAT_RGBA32F_IMAGE = 2 };
int rt_dispatch_rows_fmt(struct rt_ctx* ctx, int width, int height, int y0, int stripe, int step, int out_rows,
                         float* dst, size_t pitch, int format);

/* rt_dispatch_rows_fmt with the stripe spacing in rows: compact row r is image
 * row y0 + (r / stripe) * period + r % stripe (period >= stripe; the forms above
 * are period = stripe * step). Lets one rank own a wider stripe than the others
 * in the same period (rt_group_set_root_share). */
int rt_dispatch_rows_ex(struct rt_ctx* ctx, int width, int height, int y0, int stripe, int period, int out_rows,
                        float* dst, size_t pitch, int format);

/* glMemoryBarrier + wait: blocks until the context's stream is drained. */
int rt_sync(struct rt_ctx* ctx);

/* The wait of the reference's render loop (src/main.cpp:290-462: dispatch, barrier, draw,
 * swap): blocks until the last dispatch's frame is complete -- its image and every upload
 * issued before it. Scheduling work the renderer queued behind the frame for the next one
 * (a latency-mode cost frame's tile order) may still be running; the next dispatch on the
 * same stream runs after it. Work the host enqueued after that dispatch is not waited for
 * (use rt_sync); when there is no such frame marker it is rt_sync. */
int rt_sync_frame(struct rt_ctx* ctx);

/* Read the context surface back to host memory: `height` rows of `pitch` bytes.
 * width/height state the destination's size and must equal the surface's (the
 * last rt_dispatch's W x H), so a short buffer is refused, never overrun. */
int rt_read_image(struct rt_ctx* ctx, float* host_dst, size_t pitch, int width, int height);

/* Device pointer and pitch of the context surface (zero-copy hand-off). */
int rt_device_image(struct rt_ctx* ctx, void** ptr, size_t* pitch);

/* Runs the counting variant of the reference traversal over the same rows as
 * rt_dispatch_rows and returns the totals (synchronous; not for timed loops). */
int rt_collect_stats(struct rt_ctx* ctx, int width, int height, int y0, int stripe,
                     int step, int out_rows, rt_stats* out);
/* The same over rt_dispatch_rows_ex's rows. */
int rt_collect_stats_ex(struct rt_ctx* ctx, int width, int height, int y0, int stripe,
                        int period, int out_rows, rt_stats* out);

/* Record the device-time events around each render dispatch (default 1), which
 * rt_kernel_times / rt_last_kernel_ms read. Each is a timestamped marker on the
 * stream, and a host that waits for every frame pays for them (~4 us per waited
 * car frame, tools/group_cost.py). 0: no events; rt_kernel_times then reports
 * no dispatches. Same image either way. */
int rt_set_kernel_timing(struct rt_ctx* ctx, int on);

/* Device time of the last render kernel in ms (HIP events on the context stream). */
int rt_last_kernel_ms(struct rt_ctx* ctx, float* ms);

/* Device times (ms) of the render dispatches issued since the previous call
 * (up to 1024 are kept), written to ms[0..min(n,cap)). Returns n >= 0 and
 * restarts the record. Waits for those dispatches to finish. */
int rt_kernel_times(struct rt_ctx* ctx, float* ms, int cap);

/* Launch shape of the accelerated kernel: 1, 2 or 4 waves (8x8 tiles) per
 * workgroup; persistent != 0 = a resident grid pulling tiles from a counter. */
int rt_set_launch(struct rt_ctx* ctx, int waves_per_block, int persistent);

/* Accelerated kernel: bounces with depth >= lane_from_depth walk one ray per
 * lane (LDS stack) instead of one packet per wave; 0 = all bounces per lane,
 * >= maxBounces = all packet. Default (auto): 1 -- camera rays and their shadow
 * rays walk as packets (coherent), reflections per lane (measured fastest on
 * configs 2, 3 and 5) -- and all packets for Moller-Trumbore frames over
 * reference trees of fewer than 1024 nodes. -1 restores that automatic policy.
 * Same image for every value. */
int rt_set_walk(struct rt_ctx* ctx, int lane_from_depth);

/* Tile dispatch order of the accelerated kernel. RT_SCHED_ROWS: row-major.
 * RT_SCHED_COST (default): a dispatch records each 8x8 tile's duration (its
 * wave's wall time, in 40 ns units; every 16th frame once the order exists),
 * and the next dispatch with the same tile count starts the tiles in
 * decreasing order of those durations (longest first), so the frame is not
 * left waiting on expensive tiles that started late. The order only changes
 * when pixels are computed, never their values. RT_SCHED_COST_XCD: the same
 * longest-first order, with each bucket of equal cost split into 8 screen
 * bands, one per XCD (workgroups are dealt to the XCDs round-robin), so each
 * XCD's L2 holds the records of one band at a time. */
enum rt_schedule { RT_SCHED_ROWS = 0, RT_SCHED_COST = 1, RT_SCHED_COST_XCD = 2 };
int rt_set_schedule(struct rt_ctx* ctx, int mode);

/* Latency mode, for a host that waits for each frame before the next (the
 * reference's own loop, src/main.cpp:290-462) rather than keeping frames in
 * flight. 1: the accelerated kernel's instance with split walks in sparse
 * waves (idle lanes help a tile's few live rays) and, on frames not already
 * split, the heaviest tiles of the cost order as several waves each: 1/200 as
 * two (four for all-packet frames such as Moller-Trumbore's), and on frames of
 * few tiles per CU (a rank's share of a strong multi-GPU frame) 1/25 as eight or
 * sixteen. A dispatch whose camera moved since the last one re-ranks the tiles
 * after every frame (whole-tile wall times, each tile ranked by the largest
 * within one tile). Shortens one frame (car: -18 %) and costs throughput when
 * frames overlap. Frames of more than 12 tiles per wave slot (49,152 8x8 tiles
 * on 256 CUs: 3840x2160 has 129,600) render as in the default mode, which is
 * faster for them. 0 (default): off. Same image either way. */
int rt_set_latency_mode(struct rt_ctx* ctx, int on);

/* Ray compaction in the accelerated kernel: the rays still alive after bounce
 * from_bounce - 1 are queued per 64x64-pixel region, and a second kernel runs
 * their remaining bounces 64 rays to a wave instead of in their half-empty tile
 * waves. 0 = off; RT_TAIL_AUTO (default) = from bounce 2 on scenes whose scene
 * tree has at least 8,192 items (the 100k-triangle config: -5 %), off otherwise
 * (the car: the extra kernel costs more than it saves). Same image for every
 * value (the bounces' arithmetic is the same; a ray's walk does not depend on
 * its wave's other rays). */
enum { RT_TAIL_AUTO = -1 };
int rt_set_tail(struct rt_ctx* ctx, int from_bounce);

/* Opt-in device BVH build (lbvh.hip). Builds a linear
 * BVH (Karras 2012: Morton codes of the shapes' split() centres, radix sort,
 * one shape per leaf) on the GPU over the current shapes, in the FlatNode /
 * bvhIndices layout (root at N-1 = 2S-2, node boxes = the reference's
 * BoundingBox of their shapes), and adopts it as if the host had passed it to
 * rt_upload_scene (which also clears the animated set). It replaces the
 * reference builder's tree (src/main.cpp:1111-1193), so frames are the
 * reference shader's frames over THIS tree: read it back with rt_scene_size,
 * rt_read_nodes and rt_read_indices to reproduce them elsewhere.
 * *device_ms (optional) = device time of the build kernels. */
int rt_build_lbvh(struct rt_ctx* ctx, float* device_ms);
int rt_scene_size(struct rt_ctx* ctx, int* num_shapes, int* num_nodes, int* num_indices);
int rt_read_indices(struct rt_ctx* ctx, int* indices, int num_indices);

/* Which tree the accelerated kernel walks. RT_TREE_SCENE (default): when the
 * reference tree's child boxes nest in their parents' boxes, rays whose slab
 * values cannot be NaN walk one SAH tree over all reference leaves' shapes,
 * testing each leaf's own exact box before its shapes (the nesting makes that
 * test equivalent to the reference's walk down to the leaf); other rays walk the
 * reference tree. Animated and updated scenes keep the scene tree: the refit
 * (rt_animate, rt_update_shapes / rt_update_nodes) refits its boxes and items,
 * and node boxes that stop nesting rebuild the accelerator without it.
 * RT_TREE_REFERENCE: every ray walks the reference tree. Same image either way. */
enum rt_tree { RT_TREE_REFERENCE = 0, RT_TREE_SCENE = 1 };
int rt_set_tree(struct rt_ctx* ctx, int mode);

/* Accelerator statistics for the uploaded scene. */
int rt_accel_info_get(struct rt_ctx* ctx, rt_accel_info* out);

/* Human-readable status string. */
const char* rt_status_string(int status);

#ifdef __cplusplus
}
#endif

#endif /* RT_API_H */
