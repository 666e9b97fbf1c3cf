/*
 * rt_group.h — one frame split over several GPUs, gathered to rank 0
 * (librtamd.so).
 *
 * The reference renders a frame with one glDispatchCompute(W, H, 1) on one GPU
 * (src/main.cpp:352-354). Pixels are independent (gpu_shader.comp:434-623
 * reads no other pixel), so a group splits the frame's rows over its ranks in
 * periods of Q = share + P - 1 stripes of `stripe` rows: rank 0 renders the
 * first `share` stripes of every period, rank r >= 1 the stripe share - 1 + r.
 * With share 1 (the default) that is the interleave
 *     { image row y : (y / stripe) mod P == r }.
 * Each rank r >= 1 renders (rt_dispatch_rows_ex) into a compact packed-RGB
 * buffer (12 B per pixel: the alpha is always 1); rank 0 renders its stripes
 * straight into its pitched RGBA32F surface at their image rows
 * (RT_FORMAT_RGBA32F_IMAGE). One fan-in per frame brings the other ranks' rows
 * to rank 0 — grouped ncclSend/ncclRecv over xGMI (RCCL) or device copies — and
 * a kernel on rank 0 scatters them into image order in that surface. A group of
 * one rank renders the single-GPU frame with no fan-in and no scatter. Interleaving balances sky rows against rows through the car
 * without any per-frame planning; no other collective runs.
 *
 * Two ways to build a group:
 *  - rt_group_create: ONE process drives every device (ncclCommInitAll, the
 *    single-process plan of SURVEY §7 step 7). Devices must be distinct for
 *    RCCL; a device list with repeats uses the copy transport.
 *  - rt_group_create_rank: one process per GPU (torch.distributed.run, the
 *    bench's launch); each process holds its one member, rank `rank` of
 *    `nranks`, and the ranks meet through the 128-byte id that rank 0 makes
 *    with rt_group_unique_id and sends to the others (ncclCommInitRank).
 *
 * Frames in flight (rt_group_set_frames): each member holds F slots (a
 * context, a render stream, the frame's buffers) but ONE communicator and ONE
 * fan-in stream. Frame f renders in slot f mod F; its fan-in is queued on the
 * fan-in stream behind that render, so frame f + 1 renders while frame f
 * crosses the links, and every rank posts its sends/receives in frame order on
 * a single communicator.
 *
 * Errors. Every call returns an rt_status (rt_api.h); RT_ERR_COMM for RCCL
 * failures (and for RCCL forced on a device list with repeats). In an RCCL
 * group of more than one rank, an error inside rt_group_dispatch, an RCCL
 * asynchronous error, or an rt_group_sync that runs past the timeout aborts the
 * communicator (ncclCommAbort): peers may already have posted their half of a
 * fan-in that will never be matched. Such a group is unusable -- every later
 * call returns RT_ERR_COMM -- and every rank must destroy its group; the peers
 * see RT_ERR_COMM or RT_ERR_TIMEOUT from their own rt_group_sync.
 */
#ifndef RT_GROUP_H
#define RT_GROUP_H

#include <stddef.h>
#include "rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

struct rt_group; /* opaque */

#define RT_GROUP_ID_BYTES 128

enum rt_gather {
    RT_GATHER_AUTO = 0,  /* RCCL when the ranks' devices are distinct, copies otherwise */
    RT_GATHER_RCCL = 1,  /* ncclSend/ncclRecv to rank 0 on the members' streams          */
    RT_GATHER_COPY = 2   /* hipMemcpyPeerAsync into rank 0's staging (one process only) */
};

/* ncclGetUniqueId: rank 0 of a multi-process group makes it, every rank passes
 * it to rt_group_create_rank. `cap` >= RT_GROUP_ID_BYTES. */
int rt_group_unique_id(void* id, size_t cap);

/* One process, member k = rank k on devices[k] (n >= 1). */
int rt_group_create(struct rt_group** out, const int* devices, int n, int transport);

/* One process per GPU: this process's member is rank `rank` of `nranks`, on
 * HIP device `device`. Always RCCL (ncclCommInitRank). */
int rt_group_create_rank(struct rt_group** out, const void* id, int nranks, int rank, int device);

int rt_group_destroy(struct rt_group* g);

/* nranks, members driven by this process, transport in use (RT_GATHER_RCCL/COPY). */
int rt_group_info(struct rt_group* g, int* nranks, int* nlocal, int* transport);

/* The context of local member k (0 <= k < nlocal), for per-context settings
 * (rt_set_kernel, rt_set_walk, rt_kernel_times, ...); slot 0's with frames in
 * flight. Owned by the group. */
int rt_group_member(struct rt_group* g, int k, struct rt_ctx** ctx);
/* Member k's context of frame slot `slot` (0 <= slot < frames). */
int rt_group_member_slot(struct rt_group* g, int k, int slot, struct rt_ctx** ctx);

/* Frames in flight, 1..16 (default 1): call before rt_group_upload_scene. Frame f
 * renders in slot f mod frames. rt_group_frames returns the count. */
int rt_group_set_frames(struct rt_group* g, int frames);
int rt_group_frames(struct rt_group* g);

/* rt_upload_scene / rt_set_camera / rt_set_light / rt_set_params on every
 * local member (the scene is replicated: < 1 MB for the car, 28 MB at 100k). */
int rt_group_upload_scene(struct rt_group* g, const FlatShape* shapes, int num_shapes, const FlatNode* nodes,
                          int num_nodes, const int* indices, int num_indices);
int rt_group_set_camera(struct rt_group* g, const FlatCamera* camera);
int rt_group_set_light(struct rt_group* g, const FlatLight* light);
int rt_group_set_params(struct rt_group* g, const rt_params* params);

/* The reference's per-frame upload of an animated scene (src/main.cpp:336-346):
 * rt_update_shapes (updateScene's glBufferSubData per record, :981-992),
 * rt_update_nodes (updateBVH + serializeBVH + glBufferSubData, :340-345, :1068-1077),
 * rt_set_animated / rt_animate (the same on the device) on EVERY local member and
 * EVERY frame slot, in call order: each slot context renders every F-th frame from
 * its own copy of the scene, so each is given every frame's update (grow-only node
 * boxes need every position). Deferred or stream-ordered exactly as the
 * single-context calls (rt_api.h): one device refit per slot at its next operation.
 * The sky-row band (rt_group_set_sky_rows) follows the root box these calls leave:
 * rt_group_update_nodes sets it from node N-1, rt_group_animate grows it as the
 * device's refit grows it. Every rank must make the same calls with the same records
 * before the same frame. */
int rt_group_update_shapes(struct rt_group* g, int first, int count, const FlatShape* shapes);
int rt_group_update_nodes(struct rt_group* g, const FlatNode* nodes, int num_nodes);
int rt_group_set_animated(struct rt_group* g, const int* ids, int count);
int rt_group_animate(struct rt_group* g, const FlatShape* shapes);

/* Render the W x H frame split into `stripe`-row stripes over the ranks and
 * gather it into rank 0's surface. Stream-ordered and asynchronous; every rank
 * calls it for every frame, in the same order. */
int rt_group_dispatch(struct rt_group* g, int width, int height, int stripe);

/* Rows that can only be background stay off the links (default 1): a ray that
 * misses the root node's box draws the background of its row
 * (gpu_shader.comp:436-458), and every camera ray of an image row lies in one
 * plane through the camera, so a row whose plane has every corner of the root
 * box on one side (with a 1e-4 rad margin) is background. Each rank computes the
 * same band of rows that may meet the box from the camera, parameters and tree
 * it was given; the peers send only their rows inside it and rank 0 writes the
 * others' background (1080p car: 283 of 1080 rows). Applies to the BVH branch
 * with at least one bounce. The image does not depend on it. A member whose camera
 * or node boxes were changed through its own context (rt_group_member) instead of
 * the group's calls makes its process refuse the frame (RT_ERR_INVALID); with one
 * process per GPU the other ranks then time out in rt_group_sync and the group is
 * aborted. */
int rt_group_set_sky_rows(struct rt_group* g, int on);
/* The band [*y0, *y1) of image rows the last rt_group_dispatch sent over the links
 * ([0, height) when the band did not apply); RT_ERR_INVALID before any dispatch. */
int rt_group_sky_band(struct rt_group* g, int* y0, int* y1);

/* Rank 0's stripes per period (1 <= share <= 64; default 1). Rank 0's rows
 * never cross a link, so when rank 0's ingress bounds the frame (7 peers' rows
 * into one GPU), a larger share moves fewer bytes: of a frame's B bytes, rank 0
 * receives (P - 1) / (share + P - 1) of them. Every rank must set the same
 * value before the same frame. The image does not depend on it. */
int rt_group_set_root_share(struct rt_group* g, int share);

/* rt_collect_stats over the rows this process's members render for a
 * (width, height, stripe) frame at the current share, summed. Synchronous. */
int rt_group_collect_stats(struct rt_group* g, int width, int height, int stripe, rt_stats* out);

/* Wait until this process's members have finished every dispatched frame.
 * Bounded: it polls the streams and the communicator's asynchronous error
 * (ncclCommGetAsyncError) and gives up after the timeout (default 60 s),
 * aborting the communicator: RT_ERR_TIMEOUT, or RT_ERR_COMM on an RCCL error. */
int rt_group_sync(struct rt_group* g);
/* The timeout of rt_group_sync in ms (0 = none). */
int rt_group_set_timeout(struct rt_group* g, double ms);
/* Non-blocking: RT_ERR_COMM (and the communicator aborted) once RCCL reports an
 * asynchronous error, else RT_OK. */
int rt_group_check(struct rt_group* g);

/* Mean device times (ms) of the frames dispatched since the last call, of this
 * process's rank 0 member (else its first member), from HIP events: its stripes'
 * render, its fan-in (from the moment its stream may start it -- its own rows
 * rendered, or on rank 0 the slot free -- to the last byte sent / received, so it
 * includes waiting for the slowest peer), rank 0's unstripe, and render start to
 * the frame's last event. Waits (bounded) for the outstanding frames. */
/* Record the phase events above (default 1). 0: a frame records only the events
 * its fan-in needs (none with one rank), and rt_group_phase_times reports 0 frames. */
int rt_group_set_phase_timing(struct rt_group* g, int on);
typedef struct rt_group_phases {
    int frames;
    float render_ms, fanin_ms, unstripe_ms, frame_ms;
} rt_group_phases;
int rt_group_phase_times(struct rt_group* g, rt_group_phases* out);

/* Rank 0's surface of the LAST dispatched frame (each frame slot has its own;
 * RT_ERR_INVALID in a process without rank 0, RT_ERR_COMM once the group is
 * broken). read_image waits (bounded) and copies the whole frame; width/height
 * must equal the last dispatch's. device_image returns the surface without
 * waiting: its contents are the frame only after rt_group_sync, and stay so
 * until `frames` (rt_group_set_frames) more dispatches, which reuse the slot. */
int rt_group_read_image(struct rt_group* g, float* host_dst, size_t pitch, int width, int height);
int rt_group_device_image(struct rt_group* g, void** ptr, size_t* pitch);

#ifdef __cplusplus
}
#endif

#endif /* RT_GROUP_H */
